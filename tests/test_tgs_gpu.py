"""TGS (physx.solver_type 1, cfg/config.yaml:31) in the lane-team kernel vs the fp64 oracle's TGS restatement
(oracle/physics_oracle.c solver_type 3: position iterations as sub-steps of h / num_position_iterations, separations
advanced by J dq, a gap closing within its sub-step, a penetration pushed out over the step).
Same inputs, the one-simulate tolerances of test_physics_gpu.py through the explained-env rule, and a standing
rollout; the PGS kernels stay pinned by test_physics_gpu.py."""
import numpy as np
import pytest
import torch

from oracle.oracle import OracleSim
from tests import helpers as H

pytestmark = pytest.mark.gpu

TGS_GPU = dict(H.ANYMAL_PARAMS, solver_type=1)
TGS_ORACLE = dict(H.ANYMAL_PARAMS, solver_type=3)


@pytest.mark.parametrize("kernel", ["lane", "team"])
def test_team_tgs_one_simulate_matches_oracle(kernel, monkeypatch):
    """Both kernel forms: the lane team (gs_team.hip) and one env per lane (gs_solver.h, also the host backend's)."""
    monkeypatch.setenv("GS_PHYSICS_KERNEL", kernel)
    n = 512
    art, flat = H.anymal()
    root, dof, tau, mu = H.anymal_states(n, seed=5)
    gym, sim = H.make_gpu_sim("anymal", n, TGS_GPU)
    assert sim.kernel_variant == {"lane": 1, "team": 2}[kernel] and sim.cparams.solver_type == 1
    H.load_state_into(sim, root, dof, mu)
    sim.dof_force.copy_(torch.from_numpy(tau.astype(np.float32).reshape(-1)))
    gym.simulate(sim)
    torch.cuda.synchronize()
    g_root, g_dof = H.read_state(sim, 12)
    g_cf = sim.cf_soa.cpu().numpy().T.reshape(n, 13, 3)
    o_root, o_dof, o_cf, _ = H.oracle_run(flat, TGS_ORACLE, root, dof, tau, mu, nc=13)

    def rerun(idx, rng, bits=64):
        r, d = H.perturbed(root, dof, idx, rng)
        rr, dd, cc, _ = H.oracle_run(flat, TGS_ORACLE, r, d, tau[idx], mu[idx], bits=bits, nc=13)
        return H.state_fields(rr, dd, cc)

    H.assert_close_or_explained(H.state_fields(g_root, g_dof, g_cf), H.state_fields(o_root, o_dof, o_cf), rerun,
                                what=f"{kernel} TGS one simulate vs the oracle's TGS (512 random ANYmal states)")


def test_team_tgs_standing_rollout_tracks_oracle(monkeypatch):
    """50 env steps of PD standing (5 simulates each) under TGS: trajectories within 1e-3 of the oracle's TGS and
    visibly not the PGS trajectory's bit pattern (the mode is really on)."""
    monkeypatch.setenv("GS_PHYSICS_KERNEL", "team")
    n = 64
    art, flat = H.anymal()
    q0 = np.array([H.ANYMAL_DEFAULT[d] for d in art.dof_names()])
    root = np.zeros((n, 13)); root[:, 2] = 0.62; root[:, 6] = 1.0
    dof = np.zeros((n, 12, 2)); dof[:, :, 0] = q0
    mu = np.ones((n, flat["ns"]))
    finals = {}
    for st in (0, 1):
        gym, sim = H.make_gpu_sim("anymal", n, dict(H.ANYMAL_PARAMS, solver_type=st))
        H.load_state_into(sim, root, dof, mu)
        for step in range(50 * 5):
            g_root, g_dof = H.read_state(sim, 12)
            g_tau = np.clip(80 * (q0 - g_dof[:, :, 0]) - 2 * g_dof[:, :, 1], -80, 80)
            sim.dof_force.copy_(torch.from_numpy(g_tau.astype(np.float32).reshape(-1)))
            gym.simulate(sim)
        torch.cuda.synchronize()
        finals[st] = H.read_state(sim, 12)
    osim = OracleSim(flat, TGS_ORACLE)
    r, d = root.copy(), dof.copy()
    for step in range(50 * 5):
        tau = np.clip(80 * (q0 - d[:, :, 0]) - 2 * d[:, :, 1], -80, 80)
        osim.simulate(r, d, np.ascontiguousarray(tau), mu)
    g_root, g_dof = finals[1]
    np.testing.assert_allclose(g_root[:, 0:3], r[:, 0:3], atol=1e-3)
    np.testing.assert_allclose(g_dof[:, :, 0], d[:, :, 0], atol=1e-3)
    assert abs(g_root[:, 2].mean() - 0.49) < 0.03
    assert not np.array_equal(finals[0][0], finals[1][0])
