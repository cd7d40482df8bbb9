"""MJCF -> RawModel (host side, cold path): the subset of MuJoCo XML the in-scope assets use.

Replaces the MJCF importer inside the closed Isaac Gym binary that the reference reaches
through ``gym.load_asset(sim, root, "mjcf/nv_ant.xml", options)`` (``ant.py:149-157``).
What the reference relies on, restated from MuJoCo's documented semantics:

* ``<default>`` classes (the unnamed top-level default only): joint ``armature``,
  ``damping``, ``limited``, ``range``; geom ``density``, ``friction``, ``size``.
* ``<compiler angle="degree|radian" inertiafromgeom="true">``: joint ranges in degrees
  by default; body mass/inertia from the geoms' volumes times ``density``.
* ``<body pos quat euler>`` frames (euler in degrees with the default ``eulerseq="xyz"``,
  intrinsic), ``<freejoint>`` / ``<joint type="free">`` on the root, ``hinge`` /
  ``slide`` joints with ``axis`` and ``pos`` (the joint frame is the body frame shifted
  by ``pos``; the axis is expressed in the body frame).
* ``<geom type="sphere|capsule|box|cylinder">`` with ``pos``/``quat`` or ``fromto``;
  capsule/cylinder ``size="r half_length"`` unless ``fromto`` is given.
* ``<actuator><motor joint gear ctrlrange>``: the motor gear becomes the DOF's
  ``motor_effort`` (``ant.py:160-162`` reads it through ``get_asset_actuator_properties``).
* World-attached geoms (the floor plane) are not part of the actor.

Bodies keep document (depth-first) order; for nv_ant.xml this coincides with the
name-sorted order the URDF path uses.  Masses come out small (density 5): the Ant in the
reference is ~0.9 kg driven by 15 N m motors.
"""
from __future__ import annotations

import math
import xml.etree.ElementTree as ET
from typing import Dict, List, Optional

import numpy as np

from ._assets import (JOINT_FREE, JOINT_PRISMATIC, JOINT_REVOLUTE, SHAPE_BOX, SHAPE_CAPSULE, SHAPE_CYLINDER,
                      SHAPE_SPHERE, Pose, RawInertial, RawJoint, RawLink, RawModel, RawShape, quat_xyzw_to_mat)


def _vec(s: Optional[str], n: int, default=None):
    if s is None:
        return None if default is None else list(default)
    v = [float(x) for x in s.split()]
    if len(v) != n:
        raise ValueError(f"expected {n} numbers, got {s!r}")
    return v


def _euler_xyz_deg(e, degrees: bool) -> np.ndarray:
    a = [math.radians(x) if degrees else x for x in e]
    cx, sx, cy, sy, cz, sz = math.cos(a[0]), math.sin(a[0]), math.cos(a[1]), math.sin(a[1]), math.cos(a[2]), math.sin(a[2])
    rx = np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]])
    ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
    rz = np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]])
    return rx @ ry @ rz  # intrinsic x-y-z


def _frame(el, degrees: bool) -> Pose:
    pos = np.array(_vec(el.get("pos"), 3, [0, 0, 0]), dtype=np.float64)
    R = np.eye(3)
    if el.get("quat") is not None:
        w, x, y, z = _vec(el.get("quat"), 4)  # MuJoCo quaternions are wxyz
        n = math.sqrt(w * w + x * x + y * y + z * z)
        R = quat_xyzw_to_mat([x / n, y / n, z / n, w / n])
    elif el.get("euler") is not None:
        R = _euler_xyz_deg(_vec(el.get("euler"), 3), degrees)
    return Pose(R, pos)


def _rot_z_to(d: np.ndarray) -> np.ndarray:
    """Rotation whose z axis is the unit vector d."""
    z = d / np.linalg.norm(d)
    a = np.array([1.0, 0, 0]) if abs(z[0]) < 0.9 else np.array([0, 1.0, 0])
    x = np.cross(a, z)
    x /= np.linalg.norm(x)
    y = np.cross(z, x)
    return np.stack([x, y, z], axis=1)


# --------------------------------------------------------------- mass properties of primitives
def sphere_mass_props(r: float, rho: float):
    m = rho * 4.0 / 3.0 * math.pi * r ** 3
    return m, np.eye(3) * (0.4 * m * r * r)


def capsule_mass_props(r: float, length: float, rho: float):
    """Capsule along local z, cylinder part `length`, about its centre (hemisphere COM at 3r/8)."""
    mc = rho * math.pi * r * r * length
    mh = rho * 2.0 / 3.0 * math.pi * r ** 3  # one hemisphere
    i_axis = 0.5 * mc * r * r + 2 * (0.4 * mh * r * r)
    d = 0.5 * length + 3.0 * r / 8.0
    i_perp = mc * (r * r / 4.0 + length * length / 12.0) + 2 * (83.0 / 320.0 * mh * r * r + mh * d * d)
    return mc + 2 * mh, np.diag([i_perp, i_perp, i_axis])


def cylinder_mass_props(r: float, length: float, rho: float):
    m = rho * math.pi * r * r * length
    i_perp = m * (3 * r * r + length * length) / 12.0
    return m, np.diag([i_perp, i_perp, 0.5 * m * r * r])


def box_mass_props(size, rho: float):
    sx, sy, sz = size  # full extents
    m = rho * sx * sy * sz
    return m, np.diag([m * (sy * sy + sz * sz), m * (sx * sx + sz * sz), m * (sx * sx + sy * sy)]) / 12.0


def parse_mjcf(path: str) -> RawModel:
    root = ET.parse(path).getroot()
    comp = root.find("compiler")
    degrees = (comp.get("angle", "degree") if comp is not None else "degree") == "degree"
    from_geom = (comp.get("inertiafromgeom", "auto") if comp is not None else "auto") in ("true", "auto")
    djoint: Dict[str, str] = {}
    dgeom: Dict[str, str] = {}
    dflt = root.find("default")
    if dflt is not None:
        if dflt.find("joint") is not None:
            djoint = dict(dflt.find("joint").attrib)
        if dflt.find("geom") is not None:
            dgeom = dict(dflt.find("geom").attrib)

    gears: Dict[str, float] = {}
    act = root.find("actuator")
    if act is not None:
        for mo in act.findall("motor"):
            g = _vec(mo.get("gear"), 1, [1.0])[0] if mo.get("gear") is not None else 1.0
            cr = _vec(mo.get("ctrlrange"), 2, [-1.0, 1.0])
            gears[mo.get("joint")] = (g, max(abs(cr[0]), abs(cr[1])) if mo.get("ctrllimited", "false") == "true" else 0.0)

    links: Dict[str, RawLink] = {}
    order: List[str] = []
    joints: List[RawJoint] = []

    def geom_attr(g, k, default=None):
        return g.get(k, dgeom.get(k, default))

    def visit(be, parent_name: Optional[str], parent_frame_in_parent_link: Pose):
        name = be.get("name") or f"body{len(order)}"
        frame = _frame(be, degrees)  # body frame in the parent body frame
        shapes: List[RawShape] = []
        m_tot, c_acc, I_tot = 0.0, np.zeros(3), np.zeros((3, 3))
        parts = []
        for g in be.findall("geom"):
            gtype = geom_attr(g, "type", "sphere")
            rho = float(geom_attr(g, "density", 1000.0))
            size = _vec(geom_attr(g, "size"), len(geom_attr(g, "size").split())) if geom_attr(g, "size") else [0.0]
            ft = g.get("fromto")
            if ft is not None and gtype in ("capsule", "cylinder"):
                a, b = np.array(_vec(ft, 6)[:3]), np.array(_vec(ft, 6)[3:])
                d = b - a
                length = float(np.linalg.norm(d))
                pose = Pose(_rot_z_to(d) if length > 0 else np.eye(3), 0.5 * (a + b))
                r = size[0]
            else:
                pose = _frame(g, degrees)
                r = size[0]
                length = 2.0 * size[1] if len(size) > 1 else 0.0
            if gtype == "sphere":
                shapes.append(RawShape(SHAPE_SPHERE, pose, [r]))
                mp = sphere_mass_props(r, rho)
            elif gtype == "capsule":
                shapes.append(RawShape(SHAPE_CAPSULE, pose, [r, length]))
                mp = capsule_mass_props(r, length, rho)
            elif gtype == "cylinder":
                shapes.append(RawShape(SHAPE_CYLINDER, pose, [r, length]))
                mp = cylinder_mass_props(r, length, rho)
            elif gtype == "box":
                full = [2.0 * v for v in size]
                shapes.append(RawShape(SHAPE_BOX, pose, full))
                mp = box_mass_props(full, rho)
            else:
                continue  # planes/meshes: not part of the articulation's contact model
            parts.append((mp[0], pose.t, pose.R @ mp[1] @ pose.R.T))
        for m, c, I in parts:  # combine about the common COM (parallel axis)
            m_new = m_tot + m
            c_new = (m_tot * c_acc + m * c) / m_new if m_new > 0 else np.zeros(3)
            def shift(mi, ci, Ii):
                dd = ci - c_new
                return Ii + mi * (np.dot(dd, dd) * np.eye(3) - np.outer(dd, dd))
            I_tot = shift(m_tot, c_acc, I_tot) + shift(m, c, I) if m_tot > 0 else shift(m, c, I)
            m_tot, c_acc = m_new, c_new
        inert = RawInertial(m_tot, c_acc, I_tot) if (from_geom and m_tot > 0) else None
        ie = be.find("inertial")
        if ie is not None:
            ip = _frame(ie, degrees)
            diag = _vec(ie.get("diaginertia"), 3, [0, 0, 0])
            inert = RawInertial(float(ie.get("mass")), ip.t.copy(), ip.R @ np.diag(diag) @ ip.R.T)
        links[name] = RawLink(name, inert, shapes)
        order.append(name)

        jels = [j for j in be if j.tag in ("joint", "freejoint")]
        if parent_name is not None:
            if len(jels) != 1:
                raise ValueError(f"{path}: body {name} needs exactly one joint (has {len(jels)})")
            je = jels[0]
            jtype = je.get("type", djoint.get("type", "hinge")) if je.tag == "joint" else "free"
            kind = {"hinge": JOINT_REVOLUTE, "slide": JOINT_PRISMATIC}.get(jtype)
            if kind is None:
                raise ValueError(f"{path}: joint type {jtype} on a non-root body is not supported")
            axis = np.array(_vec(je.get("axis", djoint.get("axis")), 3, [0, 0, 1]), dtype=np.float64)
            axis /= np.linalg.norm(axis)
            jpos = np.array(_vec(je.get("pos", djoint.get("pos")), 3, [0, 0, 0]), dtype=np.float64)
            limited = je.get("limited", djoint.get("limited", "false")) == "true"
            rng = _vec(je.get("range", djoint.get("range")), 2, [0.0, 0.0])
            if kind == JOINT_REVOLUTE and degrees:
                rng = [math.radians(v) for v in rng]
            jname = je.get("name") or f"joint{len(joints)}"
            gear, ctrl = gears.get(jname, (0.0, 0.0))
            # joint frame: body frame shifted by pos; the child link frame is re-expressed so that the
            # joint sits at its origin (geoms/inertia are moved by -pos below)
            origin = Pose(parent_frame_in_parent_link.R @ frame.R,
                          parent_frame_in_parent_link.apply(frame.t + frame.R @ jpos))
            joints.append(RawJoint(name=jname, kind=kind, parent=parent_name, child=name, origin=origin, axis=axis,
                                   lower=rng[0], upper=rng[1], has_limits=limited and rng[1] > rng[0],
                                   effort=gear * ctrl if ctrl > 0 else 0.0, velocity=0.0,
                                   damping=float(je.get("damping", djoint.get("damping", 0.0))),
                                   friction=float(je.get("frictionloss", djoint.get("frictionloss", 0.0))),
                                   armature=float(je.get("armature", djoint.get("armature", 0.0))),
                                   motor_gear=gear))
            if np.any(jpos):  # move the link's content so its frame is the joint frame
                sh = Pose(np.eye(3), -jpos)
                link = links[name]
                link.shapes = [RawShape(s.kind, sh.compose(s.pose), s.size) for s in link.shapes]
                if link.inertial is not None:
                    link.inertial.com = link.inertial.com - jpos
            child_frame = Pose(np.eye(3), -jpos)
        else:
            if jels and not (jels[0].tag == "freejoint" or jels[0].get("type") == "free"):
                raise ValueError(f"{path}: the root body must be free (or have no joint)")
            child_frame = Pose()
        for cb in be.findall("body"):
            visit(cb, name, child_frame)

    wb = root.find("worldbody")
    tops = wb.findall("body")
    if len(tops) != 1:
        raise ValueError(f"{path}: expected one top-level body, found {len(tops)}")
    visit(tops[0], None, Pose())
    # default shape friction (MuJoCo geom friction[0]) for the asset's rigid shape properties
    return RawModel(root.get("model", "mjcf"), links, order, joints,
                    float(dgeom.get("friction", "1 0.005 0.0001").split()[0]))
