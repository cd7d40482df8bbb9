"""Dump a host-backend replay case for the ASan/UBSan driver (tools/asan/host_replay.cpp).

    python tools/asan/dump_case.py <out.bin> [--case hound111|hound|anymal|ant] [--n N]

The case is the r04f UsefulHound failure by default: random Hound states (seed 13, spread
0.5), actions RandomState(2), the fused 4 x PD + 1 step on the host backend.  Format (little endian): a
magic, the gs_model_desc arrays in model_desc() order (each: int64 count, int32 kind 0 int32 / 1 float64, data),
the scalar model fields, gs_sim_params, then N, nd, ns, self-collision, ground flag, the ground's frictions and
restitution, the SoA state, shape frictions, actions, default pose and
the PD gains.  The driver also writes its outputs next to it (<out.bin>.out) for compare().
"""
import argparse
import os
import struct
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from isaacgymenv_amd.isaacgym import _lib  # noqa: E402
from tests import helpers as H  # noqa: E402

MAGIC = 0x47534153  # "GSAS"


def case(name, n):
    if name.startswith("hound"):
        art, flat = H.hound()
        root, dof, _, mu = H.hound_states(256 if name == "hound111" else n, seed=13, spread=0.5)
        act = np.random.RandomState(2).uniform(-1.0, 1.0, (root.shape[0], 18))
        default = np.array([0.0, 0.7854, -1.5708] * 4 + [0.0] * 6)
        return flat, H.HOUND_PARAMS, root, dof, mu, act, default
    if name == "anymal":
        art, flat = H.anymal()
        root, dof, _, mu = H.anymal_states(n, seed=4)
        act = np.random.RandomState(0).uniform(-1, 1, (n, 12))
        default = np.array([H.ANYMAL_DEFAULT[d] for d in art.dof_names()])
        return flat, H.ANYMAL_PARAMS, root, dof, mu, act, default
    art, flat = H.ant()
    root, dof, _, mu = H.ant_states(n, seed=3)
    act = np.random.RandomState(0).uniform(-1, 1, (n, 8))
    return flat, H.ANT_PARAMS, root, dof, mu, act, np.zeros(8)


def write(path, name, n):
    """The case as the drop-in gymapi hands it to the library: the sim built by tests/helpers.make_host_sim (the
    loaded asset's model, its gs_sim_params, self-collision flag and ground), then the case's state and actions."""
    flat, params, root, dof, mu, act, default = case(name, n)
    N, nd = root.shape[0], dof.shape[1]
    gym, sim = H.make_host_sim({"hound111": "hound"}.get(name, name), N, params, threads=1)
    flat, p = sim.asset.flat, sim.cparams
    desc, keep = _lib.model_desc(flat)
    ns = int(flat["ns"])
    with open(path, "wb") as f:
        f.write(struct.pack("<I", MAGIC))
        for field, _ in _FIELDS:
            a = keep[field]
            f.write(struct.pack("<qi", a.size, 0 if a.dtype == np.int32 else 1))
            f.write(a.tobytes())
        f.write(struct.pack("<10i", desc.num_bodies, desc.num_dofs, desc.num_candidates, desc.num_shapes,
                            desc.fixed_base, desc.num_links, desc.num_hull_verts, desc.num_pairs, desc.pair_pool,
                            desc.num_pair_verts))
        f.write(struct.pack("<di3dii4dii", p.dt, p.substeps, *p.gravity, p.num_position_iterations,
                            p.num_velocity_iterations, p.contact_offset, p.rest_offset, p.bounce_threshold_velocity,
                            p.max_depenetration_velocity, p.contact_collection, p.kernel_variant))
        f.write(struct.pack("<d", p.joint_limit_margin))
        g = sim.ground
        f.write(struct.pack("<5i", N, nd, ns, int(sim.self_collide), 0 if g is None else 1))
        f.write(struct.pack("<3d", *((g.static_friction, g.dynamic_friction, g.restitution) if g is not None
                                     else (0.0, 0.0, 0.0))))
        st = np.zeros((13 + 2 * nd, N), np.float32)
        st[0:13], st[13:13 + nd], st[13 + nd:] = root.T, dof[:, :, 0].T, dof[:, :, 1].T
        f.write(st.tobytes())
        m = np.ones((ns, N), np.float32)
        m[:mu.shape[1]] = mu.T
        f.write(m.tobytes())
        f.write(np.ascontiguousarray(act, np.float32).tobytes())
        f.write(np.ascontiguousarray(default, np.float32).tobytes())
        f.write(struct.pack("<4f", 80.0, 2.0, 0.5, 80.0))
    return N, nd


# gs_model_desc pointer fields in struct order (the driver reads them back in this order)
_FIELDS = [(n, None) for n in ("parent", "joint_kind", "body_dof", "joint_origin", "joint_axis", "mass", "com",
                               "inertia", "cand_body", "cand_point", "cand_radius", "cand_shape", "dof_effort",
                               "dof_velocity", "dof_armature", "dof_lower", "dof_upper", "dof_has_limits", "cand_link",
                               "link_body", "link_pose", "link_com", "cand_dyn", "shape_kind", "shape_body",
                               "shape_link", "shape_pose", "shape_size", "shape_margin", "shape_sphere", "hull_verts",
                               "shape_hv0", "shape_hv1", "pair_a", "pair_b", "pair_kind", "pair_verts", "shape_pv0",
                               "shape_pv1")]


def compare(path, name, n):
    """The sanitized driver's outputs vs the product library's host backend on the same case."""
    import torch
    flat, params, root, dof, mu, act, default = case(name, n)
    N, nd = root.shape[0], dof.shape[1]
    gym, sim = H.make_host_sim({"hound111": "hound"}.get(name, name), N, params, threads=1)
    H.load_state_into(sim, root, dof, mu)
    gym.refresh_dof_state_tensor(sim)
    torques = torch.empty((N, nd))
    gym.amd_pd_decimation_step(sim, torch.from_numpy(act.astype(np.float32)),
                               torch.from_numpy(default.astype(np.float32)), 80.0, 2.0, 0.5, 80.0, 4, 1, torques)
    got = np.fromfile(path + ".out", np.float32)
    ref = np.concatenate([sim.state.numpy().ravel(), torques.numpy().ravel()])
    assert got.shape == ref.shape, (got.shape, ref.shape)
    assert np.all(np.isfinite(got))
    err = np.abs(got.astype(np.float64) - ref) / (1e-4 + np.abs(ref))
    return float(err.max())


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--case", default="hound111")
    ap.add_argument("--n", type=int, default=64)
    ap.add_argument("--compare", action="store_true")
    a = ap.parse_args()
    if a.compare:
        print(f"max relative difference vs the product host backend: {compare(a.out, a.case, a.n):.3g}")
    else:
        print("envs, dofs:", write(a.out, a.case, a.n))
