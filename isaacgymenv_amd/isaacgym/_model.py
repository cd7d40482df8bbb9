"""Flat (C-ABI) form of an :class:`Articulation`.

The same flat arrays feed the product library (``gs_sim_set_model`` in
``include/gymsim.h``) and, in tests, the CPU oracle.  Layout:

* ``parent[nb]``, ``jkind[nb]``, ``bdof[nb]`` (int32)
* ``jorigin[nb][12]`` -- parent body frame -> joint frame, R row-major then t
* ``jaxis[nb][3]``, ``mass[nb]``, ``com[nb][3]``, ``inertia[nb][9]`` (about COM)
* contact candidates ``cbody[nc]``, ``cpoint[nc][3]``, ``cradius[nc]``, ``cshape[nc]``
* per dof ``effort``, ``vmax``, ``armature``, ``lower``, ``upper``, ``has_limits``
* reported links (the tensor API's rigid bodies): ``nr``, ``clink[nc]`` (link whose net contact
  force a candidate adds to), ``lbody[nr]`` (dynamic body), ``lpose[nr][12]`` (link frame in the
  body frame, R row-major then t), ``lcom[nr][3]`` (link COM, link frame), ``lmass[nr]``
* ``cdyn[nc]``: hull slot of a convex hull's dynamic ground candidate (0..3), -1 for fixed points
* shapes (``Articulation.shape_table``): ``shkind``, ``shbody``, ``shlink`` [ns]; ``shpose[ns][12]`` (body
  frame); ``shsize[ns][3]``; ``shmargin[ns]``; ``shsphere[ns][4]`` (bounding sphere, body frame);
  hull vertices ``hverts[nhv][4]`` (body frame xyz, core factor f) with ``shv0``/``shv1`` [ns] ranges, and the
  self-collision core's subset ``pverts[npv][4]`` with ``shp0``/``shp1``
* self-collision pairs (``Articulation.self_collision_pairs``): ``npair``, ``pair_a``, ``pair_b``,
  ``pair_kind`` [npair]; ``npool`` self-contact slots per env
"""
from __future__ import annotations

import numpy as np

from ._assets import Articulation, JOINT_FREE, JOINT_FIXED, pair_pool_size


def flatten(art: Articulation, armature: float | None = None) -> dict:
    nb, nd = art.num_bodies, art.num_dofs
    parent = np.array([b.parent for b in art.bodies], dtype=np.int32)
    jkind = np.array([b.joint_kind for b in art.bodies], dtype=np.int32)
    bdof = np.full(nb, -1, dtype=np.int32)
    for di, d in enumerate(art.dofs):
        bdof[d.body] = di
    jorigin = np.zeros((nb, 12))
    jaxis = np.zeros((nb, 3))
    mass = np.zeros(nb)
    com = np.zeros((nb, 3))
    inertia = np.zeros((nb, 9))
    for i, b in enumerate(art.bodies):
        jorigin[i, :9] = b.origin.R.reshape(-1)
        jorigin[i, 9:] = b.origin.t
        jaxis[i] = b.axis
        mass[i] = b.mass
        com[i] = b.com
        inertia[i] = b.inertia.reshape(-1)
    cands = art.contact_candidates()
    if art.fixed_base:
        # a body welded to the world cannot take a contact impulse: drop its candidates
        cands = [c for c in cands if c[0] != 0]
    nc = len(cands)
    cbody = np.array([c[0] for c in cands], dtype=np.int32).reshape(nc)
    cpoint = np.array([c[1] for c in cands], dtype=np.float64).reshape(nc, 3)
    cradius = np.array([c[2] for c in cands], dtype=np.float64).reshape(nc)
    cshape = np.array([c[3] for c in cands], dtype=np.int32).reshape(nc)
    cdyn = np.array([c[4] for c in cands], dtype=np.int32).reshape(nc)
    clinks = art.candidate_links()
    if art.fixed_base:
        clinks = [l for l, c in zip(clinks, art.contact_candidates()) if c[0] != 0]
    clink = np.array(clinks, dtype=np.int32).reshape(nc)
    links = art.link_table()
    nr = len(links)
    lpose = np.zeros((nr, 12))
    for i, l in enumerate(links):
        lpose[i, :9] = l.pose.R.reshape(-1)
        lpose[i, 9:] = l.pose.t
    arm = art.options.get("armature", 0.0) if armature is None else armature
    tab = art.shape_table()
    ns = len(tab)
    shpose = np.zeros((ns, 12))
    hv, shv0, shv1, pv, shp0, shp1 = [], [], [], [], [], []
    for i, d in enumerate(tab):
        shpose[i, :9] = d["R"].reshape(-1)
        shpose[i, 9:] = d["t"]
        shv0.append(len(hv))
        shp0.append(len(pv))
        if d["verts"] is not None:
            hv += [list(v) + [float(f)] for v, f in zip(d["verts"], d["f"])]
            pv += [list(v) + [float(f)] for v, f in zip(d["pverts"], d["pf"])]
        shv1.append(len(hv))
        shp1.append(len(pv))
    pairs = art.self_collision_pairs() if not art.fixed_base else []
    return dict(
        nb=nb, nd=nd, nc=nc, ns=art.num_shapes, fixed_base=int(art.fixed_base),
        parent=parent, jkind=jkind, bdof=bdof, jorigin=jorigin, jaxis=jaxis, mass=mass, com=com,
        inertia=inertia, cbody=cbody, cpoint=cpoint, cradius=cradius, cshape=cshape,
        effort=np.array([d.effort for d in art.dofs], dtype=np.float64).reshape(nd),
        vmax=np.array([d.velocity for d in art.dofs], dtype=np.float64).reshape(nd),
        armature=np.array([float(arm) if d.armature is None else float(d.armature) for d in art.dofs],
                          dtype=np.float64).reshape(nd),
        lower=np.array([d.lower for d in art.dofs], dtype=np.float64).reshape(nd),
        upper=np.array([d.upper for d in art.dofs], dtype=np.float64).reshape(nd),
        has_limits=np.array([int(d.has_limits) for d in art.dofs], dtype=np.int32).reshape(nd),
        nr=nr, clink=clink, lbody=np.array([l.body for l in links], dtype=np.int32), lpose=lpose,
        lcom=np.array([l.com for l in links], dtype=np.float64).reshape(nr, 3),
        lmass=np.array([l.mass for l in links], dtype=np.float64),
        cdyn=cdyn,
        shkind=np.array([d["kind"] for d in tab], dtype=np.int32).reshape(ns),
        shbody=np.array([d["body"] for d in tab], dtype=np.int32).reshape(ns),
        shlink=np.array([d["link"] for d in tab], dtype=np.int32).reshape(ns),
        shpose=shpose, shsize=np.array([d["size"] for d in tab], dtype=np.float64).reshape(ns, 3),
        shmargin=np.array([d["margin"] for d in tab], dtype=np.float64).reshape(ns),
        shsphere=np.array([list(d["centre"]) + [d["radius"]] for d in tab], dtype=np.float64).reshape(ns, 4),
        hverts=np.array(hv, dtype=np.float64).reshape(len(hv), 4),
        shv0=np.array(shv0, dtype=np.int32).reshape(ns), shv1=np.array(shv1, dtype=np.int32).reshape(ns),
        pverts=np.array(pv, dtype=np.float64).reshape(len(pv), 4),
        shp0=np.array(shp0, dtype=np.int32).reshape(ns), shp1=np.array(shp1, dtype=np.int32).reshape(ns),
        npair=len(pairs),
        pair_a=np.array([p[0] for p in pairs], dtype=np.int32).reshape(len(pairs)),
        pair_b=np.array([p[1] for p in pairs], dtype=np.int32).reshape(len(pairs)),
        pair_kind=np.array([p[2] for p in pairs], dtype=np.int32).reshape(len(pairs)),
        npool=pair_pool_size(len(pairs)),
    )


def topology_signature(flat: dict) -> str:
    """Compile-time shape of a model: what selects a specialised kernel."""
    sig = "fb{}_p{}_c{}".format(flat["fixed_base"], "-".join(str(int(p)) for p in flat["parent"]),
                                 "-".join(str(int(b)) for b in flat["cbody"]))
    if flat["nr"] != flat["nb"] or any(int(a) != int(b) for a, b in zip(flat["clink"], flat["cbody"])):
        sig += "_l{}_{}".format(flat["nr"], "-".join(str(int(l)) for l in flat["clink"]))
    return sig
