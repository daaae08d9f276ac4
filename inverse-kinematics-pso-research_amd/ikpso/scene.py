"""Host-side scene model: the caller side of the solver boundary.

Mirrors the reference's node tree and its marshalling into the solver's
node table (src/Node.h:37-462, src/ = InverseKinematicsResearch/
InverseKinematicsResearch/):

    Node / OriginNode / EffectorNode / TargetNode   src/Node.h:45-462
    Node.to_cuda()        -> ToCUDA / CopyToArray   src/Node.h:104-108,232-267
    Node.fill_positions() -> FillPositions          src/Node.h:110-149
    Node.to_coords()      -> ToCoords / FillCoords  src/Node.h:166-194
    Node.from_coords()    -> FromCoords             src/Node.h:196-217
    check_distance()      -> checkDistance          src/Main.cpp:290-298
    reference_scene()     -> arm set-up             src/Main.cpp:76-116
    reset_arm()           -> resetArm               src/Main.cpp:330-337

Host forward kinematics here is float64 numpy (the reference uses glm float32
on the host); it is only used for the diagnostics/residual side of the caller
and for the positions[] array of the (default-off) distance term.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np

from ._abi import NODE, NODE_DTYPE, NODE_EFFECTOR, NODE_ORIGIN

PI_F = np.float32(3.14159265358979323846)  # ik_constants.h PI (a float literal)
TWO_PI_F = np.float32(2.0) * PI_F


def _rot_euler(angles) -> np.ndarray:
    a, b, c = (float(t) for t in angles)
    ca, sa, cb, sb, cc, sc = np.cos(a), np.sin(a), np.cos(b), np.sin(b), np.cos(c), np.sin(c)
    rx = np.array([[1, 0, 0, 0], [0, ca, -sa, 0], [0, sa, ca, 0], [0, 0, 0, 1]])
    ry = np.array([[cb, 0, sb, 0], [0, 1, 0, 0], [-sb, 0, cb, 0], [0, 0, 0, 1]])
    rz = np.array([[cc, -sc, 0, 0], [sc, cc, 0, 0], [0, 0, 1, 0], [0, 0, 0, 1]])
    return rx @ ry @ rz


def _translate(t) -> np.ndarray:
    m = np.eye(4)
    m[:3, 3] = [float(v) for v in t]
    return m


class TargetNode:
    """src/Node.h:375-407"""

    def __init__(self, position=(0.0, 0.0, 0.0), rotation=(0.0, 0.0, 0.0)):
        self.position = np.asarray(position, dtype=np.float32).copy()
        self.rotation = np.asarray(rotation, dtype=np.float32).copy()

    def translate(self, t):
        self.position = (self.position + np.asarray(t, dtype=np.float32)).astype(np.float32)


class Node:
    """src/Node.h:45-318: an Euler-XYZ joint followed by a link along +X."""

    node_type = NODE

    def __init__(self, rotation=(0.0, 0.0, 0.0), min_rotation=(0.0, 0.0, 0.0), max_rotation=(0.0, 0.0, 0.0),
                 length: float = 0.0, parent: Optional["Node"] = None):
        self.rotation = np.asarray(rotation, dtype=np.float32).copy()
        self.min_rotation = np.asarray(min_rotation, dtype=np.float32).copy()
        self.max_rotation = np.asarray(max_rotation, dtype=np.float32).copy()
        self.length = np.float32(length)
        self.parent = parent
        self.children: List[Node] = []
        self.effector_weight = np.float32(0.0)

    # -- tree ------------------------------------------------------------
    def attach_child(self, child: "Node") -> "Node":
        child.parent = self
        self.children.append(child)
        return child

    def dfs(self):
        yield self
        for c in self.children:
            yield from c.dfs()

    def count_children(self) -> int:
        return sum(c.count_children() + 1 for c in self.children)

    # -- host FK -----------------------------------------------------------
    def model_matrix(self) -> np.ndarray:
        """GetModelMatrix (src/Node.h:92-102)."""
        local = _rot_euler(self.rotation) @ _translate((self.length, 0.0, 0.0))
        if self.parent is None:
            return _rot_euler(self.rotation)
        return self.parent.model_matrix() @ local

    def world_position(self) -> np.ndarray:
        return (self.model_matrix() @ np.array([0.0, 0.0, 0.0, 1.0]))[:3]

    # -- marshalling -------------------------------------------------------
    def _fill_node(self, rec) -> None:
        rec["node_type"] = self.node_type

    def to_cuda(self) -> np.ndarray:
        """ToCUDA/CopyToArray: DFS order, parent index = DFS index of the parent."""
        nodes = list(self.dfs())
        index = {id(n): i for i, n in enumerate(nodes)}
        arr = np.zeros(len(nodes), dtype=NODE_DTYPE)
        for i, n in enumerate(nodes):
            rec = arr[i]
            rec["length"] = n.length
            rec["effector_weight"] = n.effector_weight
            rec["rotation"] = n.rotation
            rec["min_rotation"] = n.min_rotation
            rec["max_rotation"] = n.max_rotation
            rec["parent_index"] = -1 if n.parent is None or i == 0 else index[id(n.parent)]
            n._fill_node(rec)
        return arr

    def fill_positions(self, positions: Optional[np.ndarray] = None) -> np.ndarray:
        """FillPositions/CopyPositions: node with DFS index i writes slot (i+1)*4.
        The solver reads node k's reference position at slot (k-1)*4
        (src/kernel.cu:94-98), i.e. node k-2's -- reproduced, not fixed."""
        nodes = list(self.dfs())
        n = len(nodes)
        if positions is None:
            positions = np.zeros(4 * (n + 1), dtype=np.float32)
        for i, node in enumerate(nodes):
            p = node.model_matrix() @ np.array([0.0, 0.0, 0.0, 1.0])
            slot = (i + 1) * 4
            if slot + 4 <= positions.size:
                positions[slot:slot + 4] = p
        return positions

    def to_coords(self) -> np.ndarray:
        """ToCoords: angles of every non-origin node in DFS order."""
        return np.concatenate([n.rotation for n in list(self.dfs())[1:]]).astype(np.float32)

    def from_coords(self, coords: Sequence[float]) -> None:
        """FromCoords: inverse of to_coords."""
        coords = np.asarray(coords, dtype=np.float32)
        for i, n in enumerate(list(self.dfs())[1:]):
            n.rotation = coords[3 * i:3 * i + 3].copy()


class OriginNode(Node):
    """src/Node.h:320-373"""

    node_type = NODE_ORIGIN

    def __init__(self, position=(0.0, 0.0, 0.0), rotation=(0.0, 0.0, 0.0), min_rotation=None, max_rotation=None):
        lo = (-PI_F, -PI_F, -PI_F) if min_rotation is None else min_rotation
        hi = (PI_F, PI_F, PI_F) if max_rotation is None else max_rotation
        super().__init__(rotation, lo, hi, 0.0)
        self.position = np.asarray(position, dtype=np.float32).copy()

    def model_matrix(self) -> np.ndarray:
        return _translate(self.position) @ _rot_euler(self.rotation)

    def translate(self, t):
        self.position = (self.position + np.asarray(t, dtype=np.float32)).astype(np.float32)

    def _fill_node(self, rec) -> None:
        rec["node_type"] = NODE_ORIGIN
        rec["position"] = self.position


class EffectorNode(Node):
    """src/Node.h:409-462"""

    node_type = NODE_EFFECTOR

    def __init__(self, effector_weight: float, rotation, min_rotation, max_rotation, length: float,
                 target: Optional[TargetNode] = None, parent: Optional[Node] = None):
        super().__init__(rotation, min_rotation, max_rotation, length, parent)
        self.effector_weight = np.float32(effector_weight)
        self.target = target

    def calculate_distance(self) -> float:
        """EffectorNode::calculateDistance: |target - position|."""
        return float(np.linalg.norm(self.target.position.astype(np.float64) - self.world_position()))

    def _fill_node(self, rec) -> None:
        rec["node_type"] = NODE_EFFECTOR
        if self.target is not None:
            rec["target_position"] = self.target.position
            rec["target_rotation"] = self.target.rotation


def check_distance(effectors: Sequence[EffectorNode]) -> float:
    """checkDistance (src/Main.cpp:290-298)."""
    return float(sum(e.calculate_distance() for e in effectors))


# Reset targets (src/Main.cpp:334-336) and initial targets (src/Main.cpp:86-88).
RESET_TARGETS = np.array([[0.75, 1.0, -2.5], [-0.75, 1.0, -2.5], [0.0, 0.0, -2.5]], dtype=np.float32)
INITIAL_TARGETS = np.array([[0.5, 1.0, -2.0], [-0.5, 1.0, -2.0], [0.0, 0.0, -2.0]], dtype=np.float32)


class Scene:
    """The reference's arm (src/Main.cpp:76-116) with handles to its parts."""

    def __init__(self):
        lim_lo, lim_hi = (0.0, 0.0, 0.0), (TWO_PI_F,) * 3
        self.origin = OriginNode((0.0, 0.0, 0.0), (0.0, 0.0, 0.0), lim_lo, lim_hi)
        self.elbows = [Node((0.0, 1.57, 0.0), lim_lo, lim_hi, 1.0) for _ in range(4)]
        self.targets = [TargetNode(t) for t in INITIAL_TARGETS]
        self.effectors = [
            EffectorNode(1.0, (0.0, 1.57, 0.0), lim_lo, lim_hi, 1.0, self.targets[0]),
            EffectorNode(1.0, (0.0, 0.0, 1.57), lim_lo, lim_hi, 1.0, self.targets[1]),
            EffectorNode(1.0, (0.0, 0.0, 1.57), lim_lo, lim_hi, 1.0, self.targets[2]),
        ]
        self.origin.attach_child(self.elbows[0])
        for a, b in zip(self.elbows[:-1], self.elbows[1:]):
            a.attach_child(b)
        for e in self.effectors:
            self.elbows[-1].attach_child(e)
        self.default_coords = self.origin.to_coords()

    def reset_arm(self) -> None:
        """resetArm (src/Main.cpp:330-337)."""
        self.origin.from_coords(self.default_coords)
        for t, p in zip(self.targets, RESET_TARGETS):
            t.position = p.copy()

    def check_distance(self) -> float:
        return check_distance(self.effectors)


def reference_scene(reset: bool = True) -> Scene:
    s = Scene()
    if reset:
        s.reset_arm()
    return s


def serial_chain(joints: int, length: float, rotation=(0.0, 0.3, 0.0), lo: float = -float(PI_F),
                 hi: float = float(PI_F)) -> OriginNode:
    """Serial chain of `joints` Euler joints with a single tip effector
    (BASELINE config 5 uses 20 joints of length 0.25)."""
    origin = OriginNode((0.0, 0.0, 0.0), (0.0, 0.0, 0.0))
    parent: Node = origin
    for k in range(joints):
        if k == joints - 1:
            n = EffectorNode(1.0, rotation, (lo,) * 3, (hi,) * 3, length, TargetNode((0.0, 0.0, 0.0)))
        else:
            n = Node(rotation, (lo,) * 3, (hi,) * 3, length)
        parent = parent.attach_child(n)
    return origin


def init_colliders(count: int) -> np.ndarray:
    """initColliders (src/Main.cpp:537-559): the visualiser's first `count`
    (<= 4) unit-cube colliders, as an obj_t (COLLIDER_DTYPE) array.  The
    reference ships with colliderCount = 0 (src/Main.cpp:18)."""
    from ._abi import COLLIDER_DTYPE

    spec = [((1.0, 0.0, 0.0), (0.0, 0.0, 0.0, 1.0)),
            ((0.0, 0.0, -1.0), (-0.403, -0.819, 0.273, 0.304)),
            ((-1.0, 0.0, 0.0), (0.0, 0.0, 0.0, 1.0)),
            ((0.0, 0.0, 1.0), (0.0, 0.0, 0.0, 1.0))]
    out = np.zeros(max(0, min(int(count), 4)), dtype=COLLIDER_DTYPE)
    for i in range(out.shape[0]):
        out[i]["x"] = out[i]["y"] = out[i]["z"] = 1.0
        out[i]["pos"], out[i]["quat"] = spec[i]
    return out
