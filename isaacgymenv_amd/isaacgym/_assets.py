"""Asset import: URDF -> articulation model (host side, cold path).

Replaces the importer inside the closed Isaac Gym binary that the reference
reaches through ``gym.load_asset`` (``anymal_terrain.py:231``,
``cartpole.py:88``).  The behaviour restated here is what the reference's
callers rely on:

* ``collapse_fixed_joints`` merges every link hung on a ``fixed`` joint into
  its parent (mass, COM and inertia combined about the merged COM; collision
  shapes re-expressed in the parent frame).  AnymalTerrain relies on this to
  turn 76 URDF links into 13 bodies whose names contain ``SHANK`` (feet) and
  ``THIGH`` (knees) (``AnymalTerrain.yaml`` urdfAsset.footName/kneeName).
* bodies are ordered depth-first from the root with siblings sorted by body
  name; DOFs follow body order.  For ANYmal this gives
  ``LF_HAA, LF_HFE, LF_KFE, LH_*, RF_*, RH_*`` so that HAA joints sit at
  indices ``[0, 3, 6, 9]`` exactly as ``anymal_terrain.py:359`` assumes.
* ``replace_cylinder_with_capsule`` turns a cylinder of length L, radius r into
  a capsule whose cylindrical part has length L.
* ``fix_base_link`` pins the root body to the world.

Collision geometry is reduced to *contact candidates* for the plane contact
generator in the kernels: a sphere is one point with radius r, a capsule is its
two segment end points with radius r, a box is its 8 corners with radius 0, and a
triangle-mesh (STL) collision shape is its convex hull -- Isaac Gym's default
treatment of a mesh collider (vhacd off) -- with ALL hull vertices kept: against
the ground it has HULL_SLOTS dynamic contact slots filled every substep from the
hull vertices within contact_offset (deepest first, then the 4-point manifold
reduction of DESIGN.md 3.3), so its lowest point is exact at any orientation.

Self-collision (filter 0 actors, anymal_terrain.py:282, useful_hound.py:421): every
pair of shapes on two links that are neither the same dynamic body nor joined by a
joint (PhysX filters parent-child link pairs of an articulation) is a potential
contact pair (:meth:`Articulation.self_collision_pairs`).
"""
from __future__ import annotations

import json
import math
import os
import re
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

JOINT_FIXED, JOINT_REVOLUTE, JOINT_PRISMATIC, JOINT_FREE = 0, 1, 2, 3
SHAPE_SPHERE, SHAPE_CAPSULE, SHAPE_BOX, SHAPE_CYLINDER, SHAPE_CONVEX = 0, 1, 2, 3, 4

# ground contact slots of a convex hull (dynamic 4-point manifold over its vertices)
HULL_SLOTS = 4
# vertices of a hull's self-collision core (farthest-point sample of its vertices; the ground keeps them all):
# UsefulHound's arm hulls (16-473 vertices) lose at most 2.5 mm of their surface
HULL_PAIR_VERTS = 48


def farthest_point_sample(v: np.ndarray, n: int) -> np.ndarray:
    """Indices (ascending) of n points of v: the one farthest from the centroid, then repeatedly the point
    farthest from those chosen (first index on ties)."""
    c = v.mean(0)
    idx = [int(np.argmax(np.linalg.norm(v - c, axis=1)))]
    d = np.linalg.norm(v - v[idx[0]], axis=1)
    while len(idx) < min(n, len(v)):
        i = int(np.argmax(d))
        idx.append(i)
        d = np.minimum(d, np.linalg.norm(v - v[i], axis=1))
    return np.sort(np.array(idx, dtype=np.int64))
# pair narrowphase kinds: closed forms for sphere/capsule pairs, GJK on margin-rounded cores
PAIR_SS, PAIR_SC, PAIR_CC, PAIR_GJK = 0, 1, 2, 3
# self-contact slots per env (the pool the solver fills in pair order), per articulation size
def pair_pool_size(num_pairs: int) -> int:
    return 0 if num_pairs == 0 else (4 if num_pairs <= 64 else 8)


def read_stl(path: str) -> np.ndarray:
    """Vertices [3 * triangles, 3] of a binary or ASCII STL file."""
    with open(path, "rb") as f:
        data = f.read()
    if len(data) >= 84:
        n = int.from_bytes(data[80:84], "little")
        if 84 + 50 * n == len(data):
            rec = np.frombuffer(data[84:], dtype=np.dtype([("n", "<f4", 3), ("v", "<f4", (3, 3)), ("a", "<u2")]))
            return rec["v"].reshape(-1, 3).astype(np.float64)
    pts = [[float(x) for x in line.split()[1:4]] for line in data.decode("ascii", "replace").splitlines()
           if line.strip().startswith("vertex")]
    if not pts:
        raise ValueError(f"{path}: not an STL file")
    return np.array(pts, dtype=np.float64)


def convex_hull_vertices(vertices: np.ndarray) -> np.ndarray:
    """Every vertex of the mesh's convex hull (qhull through scipy), duplicates merged, in the order of
    their first occurrence in the mesh."""
    from scipy.spatial import ConvexHull
    _, first = np.unique(np.round(vertices, 12), axis=0, return_index=True)
    uniq = vertices[np.sort(first)]
    return uniq[np.sort(ConvexHull(uniq).vertices)]


def _mesh_file(urdf_dir: str, filename: str) -> Optional[str]:
    name = filename[len("package://"):] if filename.startswith("package://") else filename
    for base in (urdf_dir, os.path.dirname(urdf_dir)):
        p = os.path.join(base, name)
        if os.path.isfile(p):
            return p
    p = os.path.join(urdf_dir, os.path.basename(name))
    return p if os.path.isfile(p) else None


# --------------------------------------------------------------------------
# small rigid-transform helpers (float64, numpy)
# --------------------------------------------------------------------------
def rpy_to_mat(rpy) -> np.ndarray:
    r, p, y = (float(v) for v in rpy)
    cr, sr, cp, sp, cy, sy = math.cos(r), math.sin(r), math.cos(p), math.sin(p), math.cos(y), math.sin(y)
    rx = np.array([[1, 0, 0], [0, cr, -sr], [0, sr, cr]])
    ry = np.array([[cp, 0, sp], [0, 1, 0], [-sp, 0, cp]])
    rz = np.array([[cy, -sy, 0], [sy, cy, 0], [0, 0, 1]])
    return rz @ ry @ rx


def mat_to_quat_xyzw(m: np.ndarray) -> np.ndarray:
    t = np.trace(m)
    if t > 0:
        s = math.sqrt(t + 1.0) * 2
        w, x, y, z = 0.25 * s, (m[2, 1] - m[1, 2]) / s, (m[0, 2] - m[2, 0]) / s, (m[1, 0] - m[0, 1]) / s
    elif m[0, 0] > m[1, 1] and m[0, 0] > m[2, 2]:
        s = math.sqrt(1.0 + m[0, 0] - m[1, 1] - m[2, 2]) * 2
        w, x, y, z = (m[2, 1] - m[1, 2]) / s, 0.25 * s, (m[0, 1] + m[1, 0]) / s, (m[0, 2] + m[2, 0]) / s
    elif m[1, 1] > m[2, 2]:
        s = math.sqrt(1.0 + m[1, 1] - m[0, 0] - m[2, 2]) * 2
        w, x, y, z = (m[0, 2] - m[2, 0]) / s, (m[0, 1] + m[1, 0]) / s, 0.25 * s, (m[1, 2] + m[2, 1]) / s
    else:
        s = math.sqrt(1.0 + m[2, 2] - m[0, 0] - m[1, 1]) * 2
        w, x, y, z = (m[1, 0] - m[0, 1]) / s, (m[0, 2] + m[2, 0]) / s, (m[1, 2] + m[2, 1]) / s, 0.25 * s
    q = np.array([x, y, z, w])
    return q / np.linalg.norm(q)


def quat_xyzw_to_mat(q) -> np.ndarray:
    x, y, z, w = (float(v) for v in q)
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
        [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
        [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)],
    ])


@dataclass
class Pose:
    R: np.ndarray = field(default_factory=lambda: np.eye(3))
    t: np.ndarray = field(default_factory=lambda: np.zeros(3))

    def compose(self, other: "Pose") -> "Pose":
        return Pose(self.R @ other.R, self.t + self.R @ other.t)

    def apply(self, p) -> np.ndarray:
        return self.t + self.R @ np.asarray(p, dtype=np.float64)

    def to_json(self):
        return {"R": self.R.tolist(), "t": self.t.tolist()}

    @staticmethod
    def from_json(d):
        return Pose(np.array(d["R"], dtype=np.float64), np.array(d["t"], dtype=np.float64))


# --------------------------------------------------------------------------
# raw (URDF-level) description
# --------------------------------------------------------------------------
@dataclass
class RawInertial:
    mass: float = 0.0
    com: np.ndarray = field(default_factory=lambda: np.zeros(3))
    inertia: np.ndarray = field(default_factory=lambda: np.zeros((3, 3)))  # about COM, link frame axes


@dataclass
class RawShape:
    kind: int
    pose: Pose
    size: List[float]  # sphere [r]; capsule/cylinder [r, length]; box [sx, sy, sz]; convex [x, y, z, ...] points


@dataclass
class RawLink:
    name: str
    inertial: Optional[RawInertial]
    shapes: List[RawShape]
    # collision <mesh> files the importer could not read as STL (gym.load_asset warns
    # with the link names)
    dropped_meshes: List[str] = field(default_factory=list)


@dataclass
class RawJoint:
    name: str
    kind: int
    parent: str
    child: str
    origin: Pose
    axis: np.ndarray
    lower: float = 0.0
    upper: float = 0.0
    has_limits: bool = False
    effort: float = 0.0
    velocity: float = 0.0
    damping: float = 0.0
    friction: float = 0.0
    armature: Optional[float] = None   # MJCF joint armature (URDF: AssetOptions.armature)
    motor_gear: float = 0.0            # MJCF <motor gear>: the DOF's motor_effort


@dataclass
class RawModel:
    name: str
    links: Dict[str, RawLink]
    link_order: List[str]
    joints: List[RawJoint]
    default_friction: float = 1.0      # rigid shape friction the importer assigns (MJCF geom friction[0])

    # ---- (de)serialisation of the packed form shipped under assets/ ----
    def to_json(self) -> dict:
        def shp(s: RawShape):
            return {"kind": s.kind, "pose": s.pose.to_json(), "size": list(s.size)}

        links = []
        for n in self.link_order:
            l = self.links[n]
            inert = None
            if l.inertial is not None:
                inert = {"mass": l.inertial.mass, "com": l.inertial.com.tolist(),
                         "inertia": l.inertial.inertia.tolist()}
            links.append({"name": n, "inertial": inert, "shapes": [shp(s) for s in l.shapes],
                          "dropped_meshes": list(l.dropped_meshes)})
        joints = [{"name": j.name, "kind": j.kind, "parent": j.parent, "child": j.child,
                   "origin": j.origin.to_json(), "axis": j.axis.tolist(), "lower": j.lower,
                   "upper": j.upper, "has_limits": j.has_limits, "effort": j.effort,
                   "velocity": j.velocity, "damping": j.damping, "friction": j.friction,
                   "armature": j.armature, "motor_gear": j.motor_gear}
                  for j in self.joints]
        return {"format": "isaacgymenv_amd.raw_model/1", "name": self.name, "links": links, "joints": joints,
                "default_friction": self.default_friction}

    @staticmethod
    def from_json(d: dict) -> "RawModel":
        links, order = {}, []
        for l in d["links"]:
            inert = None
            if l["inertial"] is not None:
                inert = RawInertial(l["inertial"]["mass"], np.array(l["inertial"]["com"]),
                                    np.array(l["inertial"]["inertia"]))
            shapes = [RawShape(s["kind"], Pose.from_json(s["pose"]), list(s["size"])) for s in l["shapes"]]
            links[l["name"]] = RawLink(l["name"], inert, shapes, list(l.get("dropped_meshes", [])))
            order.append(l["name"])
        joints = [RawJoint(j["name"], j["kind"], j["parent"], j["child"], Pose.from_json(j["origin"]),
                           np.array(j["axis"], dtype=np.float64), j["lower"], j["upper"], j["has_limits"],
                           j["effort"], j["velocity"], j["damping"], j["friction"], j.get("armature"),
                           j.get("motor_gear", 0.0)) for j in d["joints"]]
        return RawModel(d["name"], links, order, joints, d.get("default_friction", 1.0))


_FLOAT_PREFIX = re.compile(r"^\s*[-+]?(\d+\.?\d*|\.\d+)([eE][-+]?\d+)?")


def _strtod(s: str) -> float:
    """C ``strtod`` semantics: longest valid prefix (Hound.urdf has ``0.0.0000001``)."""
    m = _FLOAT_PREFIX.match(s)
    return float(m.group(0)) if m else 0.0


def _floats(s: Optional[str], n: int, default=0.0):
    if s is None:
        return [default] * n
    v = [float(x) for x in s.split()]
    assert len(v) == n, s
    return v


def _origin(el) -> Pose:
    o = el.find("origin") if el is not None else None
    if o is None:
        return Pose()
    return Pose(rpy_to_mat(_floats(o.get("rpy"), 3)), np.array(_floats(o.get("xyz"), 3)))


def parse_urdf(path: str) -> RawModel:
    root = ET.parse(path).getroot()
    links, order = {}, []
    for le in root.findall("link"):
        name = le.get("name")
        inert = None
        ie = le.find("inertial")
        if ie is not None:
            op = _origin(ie)
            m = ie.find("mass")
            mass = float(m.get("value")) if m is not None else 0.0
            I = np.zeros((3, 3))
            ine = ie.find("inertia")
            if ine is not None:
                g = lambda k: _strtod(ine.get(k, "0"))
                I = np.array([[g("ixx"), g("ixy"), g("ixz")], [g("ixy"), g("iyy"), g("iyz")],
                              [g("ixz"), g("iyz"), g("izz")]])
            # inertia expressed in the inertial frame -> rotate into link axes
            inert = RawInertial(mass, op.t.copy(), op.R @ I @ op.R.T)
        shapes, dropped = [], []
        for ce in le.findall("collision"):
            op = _origin(ce)
            ge = ce.find("geometry")
            if ge is None:
                continue
            if ge.find("sphere") is not None:
                shapes.append(RawShape(SHAPE_SPHERE, op, [float(ge.find("sphere").get("radius"))]))
            elif ge.find("cylinder") is not None:
                c = ge.find("cylinder")
                shapes.append(RawShape(SHAPE_CYLINDER, op, [float(c.get("radius")), float(c.get("length"))]))
            elif ge.find("capsule") is not None:
                c = ge.find("capsule")
                shapes.append(RawShape(SHAPE_CAPSULE, op, [float(c.get("radius")), float(c.get("length"))]))
            elif ge.find("box") is not None:
                shapes.append(RawShape(SHAPE_BOX, op, _floats(ge.find("box").get("size"), 3)))
            elif ge.find("mesh") is not None:
                # triangle-mesh collision geometry: its convex hull's support points (STL); a file that is
                # missing or not STL is recorded so that gym.load_asset can name the links it affects
                me = ge.find("mesh")
                fn = me.get("filename", "")
                mp = _mesh_file(os.path.dirname(os.path.abspath(path)), fn)
                scale = np.array(_floats(me.get("scale"), 3, 1.0))
                try:
                    pts = convex_hull_vertices(read_stl(mp) * scale) if mp and mp.lower().endswith(".stl") else None
                except ValueError:
                    pts = None
                if pts is None:
                    dropped.append(fn)
                else:
                    shapes.append(RawShape(SHAPE_CONVEX, op, pts.reshape(-1).tolist()))
        links[name] = RawLink(name, inert, shapes, dropped)
        order.append(name)
    joints = []
    kinds = {"fixed": JOINT_FIXED, "revolute": JOINT_REVOLUTE, "continuous": JOINT_REVOLUTE,
             "prismatic": JOINT_PRISMATIC, "floating": JOINT_FREE}
    for je in root.findall("joint"):
        jt = je.get("type")
        ax = je.find("axis")
        axis = np.array(_floats(ax.get("xyz") if ax is not None else None, 3)) if ax is not None else np.array([1.0, 0, 0])
        n = np.linalg.norm(axis)
        axis = axis / n if n > 0 else np.array([1.0, 0, 0])
        lim = je.find("limit")
        dyn = je.find("dynamics")
        lower = float(lim.get("lower", 0.0)) if lim is not None else 0.0
        upper = float(lim.get("upper", 0.0)) if lim is not None else 0.0
        has_limits = jt in ("revolute", "prismatic") and lim is not None and (lim.get("lower") is not None or lim.get("upper") is not None) and upper > lower
        joints.append(RawJoint(
            name=je.get("name"), kind=kinds[jt], parent=je.find("parent").get("link"),
            child=je.find("child").get("link"), origin=_origin(je), axis=axis,
            lower=lower, upper=upper, has_limits=has_limits,
            effort=float(lim.get("effort", 0.0)) if lim is not None else 0.0,
            velocity=float(lim.get("velocity", 0.0)) if lim is not None else 0.0,
            damping=float(dyn.get("damping", 0.0)) if dyn is not None else 0.0,
            friction=float(dyn.get("friction", 0.0)) if dyn is not None else 0.0))
    name = root.get("name", os.path.basename(path))
    return RawModel(name, links, order, joints)


# --------------------------------------------------------------------------
# built articulation
# --------------------------------------------------------------------------
@dataclass
class Body:
    name: str
    parent: int
    joint_kind: int           # joint connecting to parent (JOINT_FREE / JOINT_FIXED for the root)
    joint_name: str
    origin: Pose              # parent body frame -> joint frame (at q = 0)
    axis: np.ndarray          # joint axis in the joint (= child body) frame
    mass: float
    com: np.ndarray           # in body frame
    inertia: np.ndarray       # about COM, body axes
    shapes: List[RawShape]


@dataclass
class Dof:
    name: str
    body: int
    kind: int
    lower: float
    upper: float
    has_limits: bool
    effort: float
    velocity: float
    damping: float
    friction: float
    armature: Optional[float] = None  # per-dof (MJCF); None: AssetOptions.armature
    motor_gear: float = 0.0           # MJCF motor gear (actuator motor_effort)


@dataclass
class Link:
    """A rigid body as the tensor API reports it (``collapse_fixed_joints=False`` keeps links
    hung on fixed joints).  Dynamics run on the welded :class:`Body` it belongs to."""
    name: str
    parent: int               # parent link, -1 for the root
    joint_name: str           # joint to the parent link ("" for the root)
    body: int                 # dynamic body it is welded into
    pose: "Pose"              # link frame in the body frame
    mass: float
    com: np.ndarray           # link COM in the link frame


@dataclass
class Articulation:
    name: str
    bodies: List[Body]
    dofs: List[Dof]
    fixed_base: bool
    options: dict
    default_friction: float = 1.0
    # reported rigid bodies when they differ from the dynamic bodies (fixed joints kept), else None
    links: Optional[List[Link]] = None
    # link of every shape, in shape order (None: the shape's body)
    shape_links: Optional[List[int]] = None

    @property
    def num_bodies(self):
        return len(self.bodies)

    @property
    def num_dofs(self):
        return len(self.dofs)

    def body_names(self):
        return [b.name for b in self.bodies]

    # ---- reported rigid bodies (the tensor API's view): links when fixed joints are kept
    @property
    def num_links(self):
        return len(self.links) if self.links is not None else len(self.bodies)

    def link_names(self):
        return [l.name for l in self.links] if self.links is not None else self.body_names()

    def link_table(self) -> List[Link]:
        """Every reported rigid body with its dynamic body and pose (identity when links = bodies)."""
        if self.links is not None:
            return self.links
        return [Link(b.name, b.parent, b.joint_name, i, Pose(), b.mass, b.com.copy())
                for i, b in enumerate(self.bodies)]

    def joint_names(self):
        """Joints in link order (one per non-root link, fixed joints included)."""
        return [l.joint_name for l in self.link_table()[1:]]

    def candidate_links(self) -> List[int]:
        """Reported link of every contact candidate (same order as contact_candidates())."""
        out = []
        s_index = 0
        for bi, b in enumerate(self.bodies):
            for s in b.shapes:
                link = self.shape_links[s_index] if self.shape_links is not None else bi
                n = (HULL_SLOTS if s.kind == SHAPE_CONVEX else
                     {SHAPE_SPHERE: 1, SHAPE_CAPSULE: 2, SHAPE_CYLINDER: 2, SHAPE_BOX: 8}[s.kind])
                out += [link] * n
                s_index += 1
        return out

    def shape_links_all(self) -> List[int]:
        """Reported link of every shape (shape order)."""
        out, s_index = [], 0
        for bi, b in enumerate(self.bodies):
            for _ in b.shapes:
                out.append(self.shape_links[s_index] if self.shape_links is not None else bi)
                s_index += 1
        return out

    def shape_table(self) -> List[dict]:
        """Every collision shape in the solver's terms (body frame), shape order:
        kind (0 sphere, 1 capsule, 2 box, 3 cylinder, 4 convex hull), body, link,
        pose (R, t), size (sphere [r]; capsule / cylinder [r, half length]; box half extents), margin (the
        core radius of the pair narrowphase: sphere / capsule radius; boxes, cylinders and hulls are rounded
        by m = min(0.01, a quarter of their smallest half extent)), bounding sphere (centre, radius) and,
        for hulls, the vertices (body frame) with the factor f that moves each toward the vertex centroid
        by the margin (core vertex = c + f (v - c)), and the HULL_PAIR_VERTS of them (pverts, pf) the pair
        narrowphase uses."""
        out, links = [], self.shape_links_all()
        s_index = 0
        for bi, b in enumerate(self.bodies):
            for s in b.shapes:
                d = dict(body=bi, link=links[s_index], R=s.pose.R.copy(), t=s.pose.t.copy(), verts=None, f=None,
                         pverts=None, pf=None)
                if s.kind == SHAPE_SPHERE:
                    r = float(s.size[0])
                    d.update(kind=0, size=[r, 0.0, 0.0], margin=r, centre=s.pose.t.copy(), radius=r)
                elif s.kind == SHAPE_CAPSULE:
                    r, length = (float(v) for v in s.size)
                    d.update(kind=1, size=[r, 0.5 * length, 0.0], margin=r, centre=s.pose.t.copy(),
                             radius=0.5 * length + r)
                elif s.kind == SHAPE_CYLINDER:  # (replace_cylinder_with_capsule=False): flat-ended
                    r, length = (float(v) for v in s.size)
                    d.update(kind=3, size=[r, 0.5 * length, 0.0], margin=min(0.01, 0.25 * min(r, 0.5 * length)),
                             centre=s.pose.t.copy(), radius=float(np.hypot(r, 0.5 * length)))
                elif s.kind == SHAPE_BOX:
                    h = [0.5 * float(v) for v in s.size]
                    d.update(kind=2, size=h, margin=min(0.01, 0.25 * min(h)), centre=s.pose.t.copy(),
                             radius=float(np.linalg.norm(h)))
                else:
                    v = np.array([s.pose.apply(p) for p in np.asarray(s.size, dtype=np.float64).reshape(-1, 3)])
                    c = v.mean(0)
                    dist = np.linalg.norm(v - c, axis=1)
                    half = 0.5 * (v.max(0) - v.min(0))
                    m = min(0.01, 0.25 * float(half.min()))
                    f = np.where(dist > m, 1.0 - m / np.maximum(dist, 1e-12), 0.0)
                    pi = farthest_point_sample(v, HULL_PAIR_VERTS)
                    d.update(kind=4, size=[0.0, 0.0, 0.0], margin=m, centre=c, radius=float(dist.max()),
                             R=np.eye(3), t=np.zeros(3), verts=v, f=f, pverts=v[pi], pf=f[pi])
                out.append(d)
                s_index += 1
        return out

    def self_collision_pairs(self) -> List[tuple]:
        """(shape a, shape b, kind, contact slots) for every shape pair a < b on links that may collide:
        not welded into the same dynamic body and not joined by a joint (parent-child links).  kind:
        PAIR_SS / PAIR_SC (sphere first or second) / PAIR_CC (2 slots: a parallel pair contacts at both
        ends of its overlap) / PAIR_GJK (any pair with a box, a flat-ended cylinder or a hull).
        (A cylinder's GROUND contacts stay its two end points with the radius, as before.)"""
        tab = self.shape_table()
        lt = self.link_table()
        lpar = [l.parent for l in lt]
        out = []
        for a in range(len(tab)):
            for b in range(a + 1, len(tab)):
                la, lb = tab[a]["link"], tab[b]["link"]
                if tab[a]["body"] == tab[b]["body"] or la == lb or lpar[la] == lb or lpar[lb] == la:
                    continue
                ka, kb = tab[a]["kind"], tab[b]["kind"]
                if ka == 0 and kb == 0:
                    out.append((a, b, PAIR_SS, 1))
                elif {ka, kb} == {0, 1}:
                    out.append((a, b, PAIR_SC, 1))
                elif ka == 1 and kb == 1:
                    out.append((a, b, PAIR_CC, 2))
                else:
                    out.append((a, b, PAIR_GJK, 1))
        return out

    def dof_names(self):
        return [d.name for d in self.dofs]

    def chains(self) -> List[int]:
        """Chain lengths if the tree is a 'star of chains' (root + serial branches)."""
        children = {i: [] for i in range(len(self.bodies))}
        for i, b in enumerate(self.bodies[1:], 1):
            children[b.parent].append(i)
        out = []
        for c in children[0]:
            n, cur = 1, c
            while children[cur]:
                if len(children[cur]) != 1:
                    return []
                cur = children[cur][0]
                n += 1
            out.append(n)
        return out

    def contact_candidates(self):
        """(body, local point, radius, shape index, hull slot) for every plane-contact candidate.

        Candidate order = body order, then shape order, then point order (this is
        the Gauss-Seidel order of the contact solver).  A convex hull has HULL_SLOTS
        dynamic candidates (hull slot 0..3; their point is chosen every substep from
        the hull's vertices, the stored point is the vertex centroid); every other
        candidate has hull slot -1."""
        out = []
        s_index = 0
        for bi, b in enumerate(self.bodies):
            for s in b.shapes:
                if s.kind == SHAPE_SPHERE:
                    out.append((bi, s.pose.t.copy(), s.size[0], s_index, -1))
                elif s.kind in (SHAPE_CAPSULE, SHAPE_CYLINDER):
                    r, length = s.size
                    half = 0.5 * length
                    # URDF cylinders/capsules run along the local z axis of their origin frame
                    ax = s.pose.R @ np.array([0.0, 0.0, 1.0])
                    out.append((bi, s.pose.t - half * ax, r, s_index, -1))
                    out.append((bi, s.pose.t + half * ax, r, s_index, -1))
                elif s.kind == SHAPE_BOX:
                    hx, hy, hz = (0.5 * v for v in s.size)
                    for sx in (-1, 1):
                        for sy in (-1, 1):
                            for sz in (-1, 1):
                                out.append((bi, s.pose.apply([sx * hx, sy * hy, sz * hz]), 0.0, s_index, -1))
                elif s.kind == SHAPE_CONVEX:
                    v = np.array([s.pose.apply(p) for p in np.asarray(s.size, dtype=np.float64).reshape(-1, 3)])
                    for k in range(HULL_SLOTS):
                        out.append((bi, v.mean(0), 0.0, s_index, k))
                s_index += 1
        return out

    @property
    def num_shapes(self):
        return sum(len(b.shapes) for b in self.bodies)


DEFAULT_ASSET_OPTIONS = dict(
    collapse_fixed_joints=False, replace_cylinder_with_capsule=False, fix_base_link=False,
    density=1000.0, armature=0.0, angular_damping=0.5, linear_damping=0.0, thickness=0.02,
    disable_gravity=False, default_dof_drive_mode=0, flip_visual_attachments=False,
    max_angular_velocity=64.0, max_linear_velocity=1000.0,
)


def _merge_inertial(m1, c1, I1, m2, c2, I2):
    m = m1 + m2
    if m <= 0.0:
        return 0.0, np.zeros(3), np.zeros((3, 3))
    c = (m1 * c1 + m2 * c2) / m
    def shift(mi, ci, Ii):
        d = ci - c
        return Ii + mi * (np.dot(d, d) * np.eye(3) - np.outer(d, d))
    return m, c, shift(m1, c1, I1) + shift(m2, c2, I2)


def build_articulation(raw: RawModel, options: Optional[dict] = None) -> Articulation:
    opt = dict(DEFAULT_ASSET_OPTIONS)
    if options:
        opt.update({k: v for k, v in options.items() if v is not None})
    children: Dict[str, List[RawJoint]] = {}
    child_links = set()
    for j in raw.joints:
        children.setdefault(j.parent, []).append(j)
        child_links.add(j.child)
    roots = [n for n in raw.link_order if n not in child_links]
    if len(roots) != 1:
        raise ValueError(f"asset {raw.name}: expected one root link, found {roots}")
    collapse = bool(opt["collapse_fixed_joints"])
    # collapse_fixed_joints=False with fixed joints present: the dynamics weld every fixed link into
    # its parent (a rigid weld has no dynamics of its own) while the tensor API keeps reporting each
    # link (Isaac Gym's rigid-body count, names, contact forces and Jacobian rows are per link)
    keep_links = not collapse and any(j.kind == JOINT_FIXED for j in raw.joints)
    weld = collapse or keep_links
    member_of: Dict[str, tuple] = {}
    shape_link_names: List[str] = []

    # groups: a movable body plus everything welded to it; pose of each member in the body frame
    bodies: List[Body] = []

    def make_body(link_name, parent_idx, joint: Optional[RawJoint]):
        members = [(link_name, Pose())]
        stack = [(link_name, Pose())]
        movable_children = []
        while stack:
            ln, pose = stack.pop(0)
            for j in sorted(children.get(ln, []), key=lambda jj: jj.child):
                if j.kind == JOINT_FIXED and weld:
                    p = pose.compose(j.origin)
                    members.append((j.child, p))
                    stack.append((j.child, p))
                else:
                    movable_children.append((pose, j))
        m, c, I = 0.0, np.zeros(3), np.zeros((3, 3))
        shapes = []
        idx = len(bodies)
        for ln, pose in members:
            member_of[ln] = (idx, pose)
            link = raw.links[ln]
            if link.inertial is not None and link.inertial.mass > 0:
                mi = link.inertial.mass
                ci = pose.apply(link.inertial.com)
                Ii = pose.R @ link.inertial.inertia @ pose.R.T
                m, c, I = _merge_inertial(m, c, I, mi, ci, Ii)
            for s in link.shapes:
                kind = s.kind
                if kind == SHAPE_CYLINDER and opt["replace_cylinder_with_capsule"]:
                    kind = SHAPE_CAPSULE
                shapes.append(RawShape(kind, pose.compose(s.pose), list(s.size)))
                shape_link_names.append(ln)
        if joint is None:
            kind = JOINT_FIXED if opt["fix_base_link"] else JOINT_FREE
            b = Body(link_name, -1, kind, "", Pose(), np.array([1.0, 0, 0]), m, c, I, shapes)
        else:
            b = Body(link_name, parent_idx, joint.kind, joint.name, joint.origin, joint.axis.copy(), m, c, I, shapes)
        bodies.append(b)
        # children visited depth-first, siblings sorted by body name
        for pose, j in sorted(movable_children, key=lambda pj: pj[1].child):
            jj = RawJoint(**{**j.__dict__, "origin": pose.compose(j.origin)})
            make_body(j.child, idx, jj)
        return idx

    make_body(roots[0], -1, None)
    dofs = []
    for bi, b in enumerate(bodies[1:], 1):
        if b.joint_kind in (JOINT_REVOLUTE, JOINT_PRISMATIC):
            j = next(jj for jj in raw.joints if jj.name == b.joint_name)
            dofs.append(Dof(j.name, bi, j.kind, j.lower, j.upper, j.has_limits, j.effort, j.velocity,
                            j.damping, j.friction, j.armature, j.motor_gear))
    # bodies with no mass get a tiny inertia from density over their shapes' volume (Isaac Gym uses
    # `density` for links that declare no inertial); keep M non-singular
    for b in bodies:
        if b.mass <= 0.0:
            b.mass = 1e-3
            b.inertia = np.eye(3) * 1e-6
        else:
            # guard zero rotational inertia (e.g. cartpole pole declares mass only)
            ev = np.linalg.eigvalsh(b.inertia) if np.any(b.inertia) else np.zeros(3)
            if ev.min() <= 0.0:
                b.inertia = b.inertia + np.eye(3) * max(1e-6, 1e-4 * b.mass * 0.01)
    links, shape_links = None, None
    if keep_links:
        links = []
        parent_joint = {j.child: j for j in raw.joints}

        def visit(ln, parent_link):
            bi, pose = member_of[ln]
            inert = raw.links[ln].inertial
            li = len(links)
            j = parent_joint.get(ln)
            links.append(Link(ln, parent_link, j.name if j is not None else "", bi, pose,
                              float(inert.mass) if inert is not None else 0.0,
                              inert.com.copy() if inert is not None else np.zeros(3)))
            for jj in sorted(children.get(ln, []), key=lambda x: x.child):
                visit(jj.child, li)

        visit(roots[0], -1)
        index = {l.name: i for i, l in enumerate(links)}
        shape_links = [index[n] for n in shape_link_names]
        # Isaac Gym numbers DOFs in link order: the welded tree must give the same order
        link_dofs = [l.joint_name for l in links[1:] if parent_joint[l.name].kind != JOINT_FIXED]
        if link_dofs != [d.name for d in dofs]:
            raise ValueError(f"asset {raw.name}: welded DOF order {[d.name for d in dofs]} differs from the "
                             f"link order {link_dofs}")
    return Articulation(raw.name, bodies, dofs, bool(opt["fix_base_link"]), opt, raw.default_friction,
                        links, shape_links)


# --------------------------------------------------------------------------
# packed models shipped in-tree (the reference assets are not on the GPU box)
# --------------------------------------------------------------------------
PACKED_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets")
PACKED_INDEX = {
    "anymal_minimal.urdf": "anymal_c.model.json",
    "cartpole.urdf": "cartpole.model.json",
    "Hound.urdf": "hound.model.json",
    "nv_ant.xml": "nv_ant.model.json",
    # (keyed by the last two path components where a file name is shared: hound.py loads urdf/Hound_new/Hound.urdf,
    # useful_hound.py urdf/UsefulHound/urdf/Hound.urdf)
    "Hound_new/Hound.urdf": "hound_new.model.json",
}


def load_raw(root: str, filename: str) -> RawModel:
    path = os.path.join(root, filename)
    base = os.path.basename(filename)
    if os.path.isfile(path) and path.endswith(".urdf"):
        return parse_urdf(path)
    if os.path.isfile(path) and path.endswith(".xml"):
        from . import _mjcf
        return _mjcf.parse_mjcf(path)
    key2 = "/".join(filename.replace(os.sep, "/").split("/")[-2:])
    for key in (key2, base):
        if key in PACKED_INDEX:
            with open(os.path.join(PACKED_DIR, PACKED_INDEX[key])) as f:
                return RawModel.from_json(json.load(f))
    raise FileNotFoundError(f"asset not found: {path} (and no packed model named {base})")
