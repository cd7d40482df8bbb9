"""The headline fused step against the fp64 oracle at the bench config.

``gs_sim_pd_step`` (one kernel: 4 PD evaluations + 5 simulates, reference
anymal_terrain.py:441-451 pre_physics_step + vec_task.py's control_freq_inv simulate) runs on
AnymalTerrain at 4096 envs, plane, from states reached by 20 random-action env steps (resets
included).  The oracle replays the same sequence in fp64: the first PD torque from the stale dof
tensor (refreshed after the 4th simulate of the previous step, not after the 5th), the next three
from the oracle's own state, the 5th simulate with the last torque.

Every env is compared (final sim state, the dof tensor written after the 4th simulate, the torques,
the last substep's net contact forces).  An env beyond the tolerance must be explained: the oracle
itself, started from the same state perturbed at fp32-rounding size, has to move that env by at
least half the tolerance (a contact switching activity or friction regime on a last-bit difference).
The worst env is reported either way; no unexplained env is allowed.
"""
import numpy as np
import pytest
import torch

from oracle.oracle import OracleSim
from tests import helpers as H

pytestmark = pytest.mark.gpu

N = 4096
# tolerances of 5 substeps (test_physics_gpu.py bounds one substep at 2e-5 / 5e-3)
TOL = {"q": (1e-4, 0.0), "qd": (2.5e-2, 2.5e-2), "pose": (1e-4, 0.0), "vel": (2.5e-2, 2.5e-2),
       "dof_out_q": (1e-4, 0.0), "dof_out_qd": (2.5e-2, 2.5e-2), "tau": (0.5, 1e-2), "cf": (2.0, 5e-2)}


def _make(monkeypatch):
    from isaacgymenv_amd.isaacgymenvs.tasks.base import vec_task
    monkeypatch.setattr(vec_task, "EXISTING_SIM", None)
    import isaacgymenvs
    torch.manual_seed(42)
    return isaacgymenvs.make(seed=42, task="AnymalTerrain", num_envs=N, sim_device="cuda:0", rl_device="cuda:0",
                             headless=True, force_render=False)


def _oracle_sequence(flat, root, dof, dof_tensor, mu, act, default, kp, kd, scale, decimation=4, extra=1):
    """anymal_terrain.py:443-451 then vec_task's extra simulate, in fp64."""
    sim = OracleSim(flat, H.ANYMAL_PARAMS)
    r, d = root.copy(), dof.copy()
    cf = np.zeros((root.shape[0], flat["nb"], 3))
    q, qd = dof_tensor[:, :, 0], dof_tensor[:, :, 1]
    dof_out = tau = None
    for i in range(decimation + extra):
        if i < decimation:
            tau = np.clip(kp * (scale * act + default - q) - kd * qd, -80.0, 80.0)
        sim.simulate(r, d, np.ascontiguousarray(tau), mu, cf)
        q, qd = d[:, :, 0].copy(), d[:, :, 1].copy()
        if i == decimation - 1:
            dof_out = d.copy()
    return dict(q=d[:, :, 0], qd=d[:, :, 1], pose=r[:, :7], vel=r[:, 7:], dof_out_q=dof_out[:, :, 0],
                dof_out_qd=dof_out[:, :, 1], tau=tau, cf=cf)


def _ratio(a, b, key):
    atol, rtol = TOL[key]
    err = np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64))
    tol = atol + rtol * np.abs(np.asarray(b, np.float64))
    return (err / tol).reshape(err.shape[0], -1).max(axis=1), err.reshape(err.shape[0], -1).max(axis=1)


def test_fused_headline_step_matches_oracle_at_bench_config(monkeypatch):
    env = _make(monkeypatch)
    gen = torch.Generator(device="cuda:0").manual_seed(11)
    for _ in range(20):
        env.step(2 * torch.rand((N, 12), device="cuda:0", generator=gen) - 1)
    torch.cuda.synchronize()
    art, flat = H.anymal()
    assert env.sim.kernel_variant == 2, "the bench config runs the lane-team kernel"
    root, dof = H.read_state(env.sim, 12)
    dof_tensor = env.dof_state.view(N, 12, 2).double().cpu().numpy()
    mu = np.ascontiguousarray(env.sim.shape_mu.cpu().numpy().T[:, :flat["ns"]], dtype=np.float64)
    act_t = (2 * torch.rand((N, 12), device="cuda:0", generator=gen) - 1).contiguous()
    act = act_t.double().cpu().numpy()
    default_row = env.default_dof_pos[0].contiguous()
    default = default_row.double().cpu().numpy()
    kp, kd, scale = float(env.Kp), float(env.Kd), float(env.action_scale)
    torques = torch.empty((N, 12), device="cuda:0")

    env.gym.amd_pd_decimation_step(env.sim, act_t, default_row, kp, kd, scale, 80.0, env.decimation,
                                   env.control_freq_inv, torques)
    torch.cuda.synchronize()
    g_root, g_dof = H.read_state(env.sim, 12)
    g_dof_out = env.dof_state.view(N, 12, 2).double().cpu().numpy()
    gpu = dict(q=g_dof[:, :, 0], qd=g_dof[:, :, 1], pose=g_root[:, :7], vel=g_root[:, 7:],
               dof_out_q=g_dof_out[:, :, 0], dof_out_qd=g_dof_out[:, :, 1],
               tau=torques.double().cpu().numpy(), cf=env.contact_forces.double().cpu().numpy())
    assert all(np.all(np.isfinite(v)) for v in gpu.values())

    ref = _oracle_sequence(flat, root, dof, dof_tensor, mu, act, default, kp, kd, scale, env.decimation,
                           env.control_freq_inv)
    ratio = np.zeros(N)
    worst_field = np.array([""] * N, dtype=object)
    for key in TOL:
        r, _ = _ratio(gpu[key], ref[key], key)
        upd = r > ratio
        worst_field[upd] = key
        ratio = np.maximum(ratio, r)
    off = np.nonzero(ratio > 1.0)[0]

    # the oracle's own sensitivity at the diverging envs: fp32-rounding-sized perturbations of the start
    spread = np.zeros(N)
    if off.size:
        rng = np.random.RandomState(0)
        sub = lambda x: x[off]  # noqa: E731
        for _ in range(4):
            pr, pd_ = root[off].copy(), dof[off].copy()
            pr[:, :3] += rng.normal(0, 1e-6, (off.size, 3))
            pr[:, 7:] += rng.normal(0, 1e-5, (off.size, 6))
            pd_[:, :, 0] += rng.normal(0, 1e-6, (off.size, 12))
            pd_[:, :, 1] += rng.normal(0, 1e-5, (off.size, 12))
            per = _oracle_sequence(flat, pr, pd_, dof_tensor[off], mu[off], act[off], default, kp, kd, scale,
                                   env.decimation, env.control_freq_inv)
            for key in TOL:
                r, _ = _ratio(per[key], sub(ref[key]), key)
                spread[off] = np.maximum(spread[off], r)
    unexplained = off[spread[off] < 0.5]
    w = int(np.argmax(ratio))
    report = (f"worst env {w}: {ratio[w]:.3g} x tolerance in {worst_field[w]} (oracle spread {spread[w]:.3g}); "
              f"{off.size} of {N} envs beyond tolerance, {unexplained.size} unexplained")
    print(report)
    assert unexplained.size == 0, report + f"; unexplained envs {unexplained[:10].tolist()} " \
        f"({[worst_field[i] for i in unexplained[:10]]}, ratios {np.round(ratio[unexplained[:10]], 2).tolist()})"
    # a contact-switch env is rare at this state mix; a systematic error would make many envs "sensitive"
    assert off.size <= 0.02 * N, report
