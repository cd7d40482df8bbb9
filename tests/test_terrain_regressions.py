"""Trimesh contact-rule regressions replayed from captured GPU states (tests/golden/trimesh_*_case.npz,
captured by tools/probes/trimesh_nan_capture.py on an MI355X from the AnymalTerrain trimesh task).

trimesh_inverted_face_case.npz: one env-step (4 PD evaluations + 5 substeps) of an ANYmal whose knee
candidate reached, from inside the terrain, the back of a triangle the slope-threshold vertex moves had
inverted (face normal z = -0.75).  The face-from-behind rule admitted it at -0.18 m and the push-out
launched the robot (base angular velocity 2 -> 33 rad/s in one step; NaN a few hundred steps later,
which then reached the PPO learner).  Downward-facing triangles no longer generate contacts (DESIGN.md
3.7): the step stays smooth, on the host backend (the product solver source) and on the GPU, and both
agree with the fp64 oracle.
"""
import os

import numpy as np
import pytest
import torch

from tests import helpers as H

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _replay(host: bool):
    from isaacgymenv_amd.isaacgym import gymtorch
    d = np.load(os.path.join(GOLDEN, "trimesh_inverted_face_case.npz"))
    ox, oy = (float(v) for v in d["patch_origin"])
    ter = H.terrain_from_heights(d["hpatch"], hs=float(d["hs"]), vs=float(d["vs"]),
                                 slope_threshold=float(d["slope_threshold"]), shift=(ox, oy, 0.0),
                                 friction=float(d["terrain_mu"]))
    params = dict(dt=float(d["dt"]), substeps=int(d["substeps"]), gravity=[0.0, 0.0, -9.81],
                  pos_iters=int(d["pos_iters"]), vel_iters=int(d["vel_iters"]),
                  contact_offset=float(d["contact_offset"]), rest_offset=float(d["rest_offset"]),
                  max_depen_vel=float(d["max_depen"]), collect_contacts=1, has_ground=0)
    gym, sim = H.make_gpu_sim("anymal", 1, params, terrain=ter, host=host, threads=1)
    dev = "cpu" if host else "cuda:0"
    root_t = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    dof_t = gymtorch.wrap_tensor(gym.acquire_dof_state_tensor(sim))
    root_t.copy_(torch.from_numpy(d["root"]).view(1, 13))
    gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root_t))
    dof_t.copy_(torch.from_numpy(d["dof_true"]).view(-1, 2))
    gym.set_dof_state_tensor(sim, gymtorch.unwrap_tensor(dof_t))
    sim.shape_mu.copy_(torch.from_numpy(d["shape_mu"]).view(-1, 1))
    internal0 = sim.state.cpu().numpy().astype(np.float64)
    a = torch.from_numpy(d["actions"]).to(dev)
    dflt = torch.from_numpy(d["default_dof_pos"]).to(dev)
    kp, kd, sc = float(d["kp"]), float(d["kd"]), float(d["action_scale"])
    dof_for_pd = torch.from_numpy(d["dof_stale"]).to(dev)
    taus = []
    for it in range(int(d["decimation"]) + 1):
        if it < int(d["decimation"]):  # the first PD evaluation reads the task's stale dof tensor
            tau = torch.clamp(kp * (sc * a + dflt - dof_for_pd[:, 0]) - kd * dof_for_pd[:, 1], -80.0, 80.0)
        taus.append(tau.cpu().numpy().astype(np.float64).reshape(1, -1))
        sim.dof_force.copy_(tau.reshape(-1))
        gym.simulate(sim)
        gym.refresh_dof_state_tensor(sim)
        dof_for_pd = dof_t.view(12, 2).clone()
    root, dof = H.read_state(sim, 12)
    return d, ter, params, internal0, taus, root, dof


def _oracle(ter, params, internal0, taus, shape_mu):
    from oracle.oracle import OracleSim
    art, flat = H.anymal()
    osim = OracleSim(flat, params, terrain=ter["oracle"])
    r = internal0[0:13].T.copy()
    q = np.stack([internal0[13:25].T, internal0[25:37].T], axis=-1)
    mu = np.asarray(shape_mu, dtype=np.float64).reshape(1, -1)
    cf = np.zeros((1, flat["nb"], 3))
    for tau in taus:
        osim.simulate(r, q, np.ascontiguousarray(tau), mu, cf)
    return r, q


def _check(host):
    d, ter, params, internal0, taus, root, dof = _replay(host)
    w = np.linalg.norm(root[0, 10:13])
    v = np.linalg.norm(root[0, 7:10])
    assert np.isfinite(root).all() and w < 5.0 and v < 2.0, (w, v)  # was 33 rad/s, 7.5 m/s
    r, q = _oracle(ter, params, internal0, taus, d["shape_mu"])
    np.testing.assert_allclose(root[0, :3], r[0, :3], atol=2e-4)
    np.testing.assert_allclose(root[0, 7:13], r[0, 7:13], atol=2e-2, rtol=2e-2)
    np.testing.assert_allclose(dof[0, :, 0], q[0, :, 0], atol=2e-4)


def test_inverted_face_case_host_backend():
    _check(host=True)


@pytest.mark.gpu
def test_inverted_face_case_gpu():
    _check(host=False)
