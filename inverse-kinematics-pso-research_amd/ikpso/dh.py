"""Denavit-Hartenberg front-end: a serial arm given by DH parameters, mapped
onto the reference's node model.

The reference's node (src/Node.h:92-102, solver FK src/kernel.cu:31-62) is an
Euler joint followed by a link along its local +X:

    M_k = M_parent(k) * Rx(x_k) * Ry(y_k) * Rz(z_k) * T(length_k, 0, 0)

and an axis is locked by giving it equal clamp bounds (the clamp,
src/matrix_operations.cuh:187-190, pins it; the angle term then sees
x = rest).  A standard (distal) DH joint

    A_i = Rz(theta_i) * Tz(d_i) * Tx(a_i) * Rx(alpha_i)

maps onto ONE node when d_i = 0: the fixed part carried in from the previous
joint, K_i = Rx(p) Ry(q) Rz(r), is merged with the joint's Rz(theta_i) into
Rx(p) Ry(q) Rz(r + theta_i) (x and y locked, z free within the joint limits
shifted by r) and the link is T(a_i, 0, 0); Rx(alpha_i) commutes with Tx and
becomes the next joint's K.  When d_i != 0 the offset (a_i, 0, d_i) is not
along +X: the joint node gets length 0 and a locked node Ry(beta) with length
|(a_i, d_i)| follows (beta = atan2(-d_i, a_i) turns +X onto the offset), whose
inverse is folded into the next K.  The last node is the tool effector.

The chain then runs through the same solver kernels as any reference scene;
serial chains of 6, 7 and 20 nodes with a tip effector have specialised
kernels.  Joint angles map back as theta_i = z_node - r_i.

With the joint-axis mask (`DHArm.axis_mask`, ABI >= 4) only the joint nodes' z
angles are PSO dimensions: D = number of joints, locked angles take no draws
and no update, and a FAST solver folds the arm into one sincos per joint
(TopoDH, include/ikpso.h).  Without it every locked angle is emulated by equal
clamp bounds and still costs draws, an update and a sincos (3 per node).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

from .scene import EffectorNode, Node, OriginNode, TargetNode


# KUKA LBR iiwa 14 R820 (standard DH; lengths in m, joint limits in rad): the
# 7-joint arm the DH tests and bench.py --config dh7 use.
IIWA14 = dict(a=[0.0] * 7, alpha=[-np.pi / 2, np.pi / 2, np.pi / 2, -np.pi / 2, -np.pi / 2, np.pi / 2, 0.0],
              d=[0.36, 0.0, 0.42, 0.0, 0.4, 0.0, 0.126],
              limits=np.radians([170.0, 120.0, 170.0, 120.0, 170.0, 120.0, 175.0]))


def _rx(a):
    c, s = np.cos(a), np.sin(a)
    return np.array([[1, 0, 0], [0, c, -s], [0, s, c]])


def _ry(a):
    c, s = np.cos(a), np.sin(a)
    return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])


def _rz(a):
    c, s = np.cos(a), np.sin(a)
    return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])


def euler_xyz(r: np.ndarray):
    """(p, q, r) with R = Rx(p) Ry(q) Rz(r) (the reference's rotateEuler order)."""
    sq = float(np.clip(r[0, 2], -1.0, 1.0))
    q = np.arcsin(sq)
    if abs(sq) < 1.0 - 1e-12:
        p = np.arctan2(-r[1, 2], r[2, 2])
        z = np.arctan2(-r[0, 1], r[0, 0])
    else:  # gimbal lock: put everything in z
        p = 0.0
        z = np.arctan2(r[1, 0], r[1, 1])
    return float(p), float(q), float(z)


def dh_matrix(theta, d, a, alpha) -> np.ndarray:
    """Standard DH link transform Rz(theta) Tz(d) Tx(a) Rx(alpha) (float64 4x4)."""
    ct, st, ca, sa = np.cos(theta), np.sin(theta), np.cos(alpha), np.sin(alpha)
    return np.array([[ct, -st * ca, st * sa, a * ct],
                     [st, ct * ca, -ct * sa, a * st],
                     [0.0, sa, ca, d],
                     [0.0, 0.0, 0.0, 1.0]])


def dh_forward(theta: Sequence[float], d, a, alpha, base: Optional[np.ndarray] = None) -> np.ndarray:
    """Tool position of a standard DH arm (float64), the textbook product."""
    m = np.eye(4) if base is None else np.asarray(base, dtype=np.float64)
    for t, di, ai, al in zip(theta, d, a, alpha):
        m = m @ dh_matrix(t, di, ai, al)
    return m[:3, 3]


@dataclass
class DHArm:
    """A DH arm built as a reference node tree.  `origin` is the tree's root
    (marshal it with origin.to_cuda()); `joint_nodes[i]` carries theta_i in its
    z angle, offset by `z_offset[i]`; `tool` is the effector node."""

    origin: OriginNode
    joint_nodes: List[Node]
    z_offset: np.ndarray
    tool: EffectorNode
    target: TargetNode

    @property
    def dof(self) -> int:
        """Scalar angles of the node table (3 per node, most locked)."""
        return 3 * self.origin.count_children()

    @property
    def joints(self) -> int:
        """DH joints = the free dimensions under `axis_mask`."""
        return len(self.joint_nodes)

    @property
    def axis_mask(self) -> np.ndarray:
        """Joint-axis mask of the node table ([node_count] uint8, bit c = Euler
        angle c free): each joint node's z angle, nothing else."""
        ids = {id(n) for n in self.joint_nodes}
        nodes = list(self.origin.dfs())
        return np.array([0] + [4 if id(n) in ids else 0 for n in nodes[1:]], dtype=np.uint8)

    def joint_angles(self, coords: np.ndarray) -> np.ndarray:
        """theta per DH joint from a solver angle vector: ToCoords order (3 per
        node), or the masked solver's D = joints free angles."""
        coords = np.asarray(coords, dtype=np.float64).reshape(-1)
        if coords.size == self.joints:
            return coords - self.z_offset
        coords = coords.reshape(-1, 3)
        nodes = list(self.origin.dfs())[1:]
        idx = {id(n): i for i, n in enumerate(nodes)}
        return np.array([coords[idx[id(n)], 2] for n in self.joint_nodes]) - self.z_offset

    def coords(self, theta: Sequence[float], masked: bool = False) -> np.ndarray:
        """Solver angle vector for joint angles theta: ToCoords order, or with
        `masked` the D = joints free angles of the axis-masked solver."""
        if masked:
            return (np.asarray(theta, dtype=np.float64) + self.z_offset).astype(np.float32)
        nodes = list(self.origin.dfs())[1:]
        out = np.concatenate([n.rotation for n in nodes]).astype(np.float64).reshape(-1, 3)
        idx = {id(n): i for i, n in enumerate(nodes)}
        for n, t, r in zip(self.joint_nodes, theta, self.z_offset):
            out[idx[id(n)], 2] = r + t
        return out.ravel().astype(np.float32)


def dh_arm(a: Sequence[float], alpha: Sequence[float], d: Sequence[float], theta_lo: Sequence[float],
           theta_hi: Sequence[float], theta_rest: Optional[Sequence[float]] = None,
           target=(0.0, 0.0, 0.0), base_position=(0.0, 0.0, 0.0)) -> DHArm:
    """Build the node tree of a standard-DH serial arm (see the module doc)."""
    n = len(a)
    if not (len(alpha) == len(d) == len(theta_lo) == len(theta_hi) == n) or n == 0:
        raise ValueError("DH parameter lists must have one entry per joint")
    rest = np.zeros(n) if theta_rest is None else np.asarray(theta_rest, dtype=np.float64)
    origin = OriginNode(base_position, (0.0, 0.0, 0.0), (0.0, 0.0, 0.0), (0.0, 0.0, 0.0))
    tgt = TargetNode(target)
    parent: Node = origin
    k = np.eye(3)  # fixed rotation carried into the next joint
    joints, offsets = [], []
    tool = None
    for i in range(n):
        p, q, r = euler_xyz(k)
        last_joint = i == n - 1
        has_d = float(d[i]) != 0.0
        length = 0.0 if has_d else float(a[i])
        rot = (p, q, r + rest[i])
        lo = (p, q, r + float(theta_lo[i]))
        hi = (p, q, r + float(theta_hi[i]))
        if last_joint and not has_d:
            node = EffectorNode(1.0, rot, lo, hi, length, tgt)
            tool = node
        else:
            node = Node(rot, lo, hi, length)
        parent = parent.attach_child(node)
        joints.append(node)
        offsets.append(r)
        if has_d:
            beta = float(np.arctan2(-float(d[i]), float(a[i])))
            ln = float(np.hypot(float(a[i]), float(d[i])))
            fixed = (0.0, beta, 0.0)
            if last_joint:
                node = EffectorNode(1.0, fixed, fixed, fixed, ln, tgt)
                tool = node
            else:
                node = Node(fixed, fixed, fixed, ln)
            parent = parent.attach_child(node)
            k = _ry(-beta) @ _rx(float(alpha[i]))
        else:
            k = _rx(float(alpha[i]))
    return DHArm(origin, joints, np.asarray(offsets, dtype=np.float64), tool, tgt)


def iiwa14(target=(0.0, 0.0, 0.0)) -> DHArm:
    """The IIWA14 arm as a node tree (joint limits +-limits)."""
    lim = IIWA14["limits"]
    return dh_arm(IIWA14["a"], IIWA14["alpha"], IIWA14["d"], -lim, lim, target=target)
