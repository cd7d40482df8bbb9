"""Physics parity at the BASELINE.json sizes: one ``gym.simulate`` of the Ant and the
UsefulHound GPU kernels against the fp64 oracle at 4096 envs, from states the tasks themselves reached.

* Ant (BASELINE config 2; ant.py:281-297): ``isaacgymenvs.make(task=Ant, num_envs=4096)`` stepped 30 times with
  random actions (resets included), then one simulate of the one-env-per-lane kernel (Topo_nv_ant: 2 substeps,
  joint-limit rows, the four foot force sensors) with the task's own next torques.
* UsefulHound (BASELINE config 4; useful_hound.py:695-760): ``make(task=UsefulHound, num_envs=4096)`` stepped
  30 times, then one simulate of the split self-collision form (k_pair_records + k_simulate<Topo_hound>) with
  random leg and arm efforts.

Every env is within the one-simulate tolerances of DESIGN.md section 4 or explained by the oracle's own spread
(helpers.assert_close_or_explained, at most 2 % explained).  The reports go to $PARITY_REPORT.
"""
import numpy as np
import pytest
import torch

from tests import helpers as H

pytestmark = pytest.mark.gpu

N = 4096
# the one-simulate tolerances with the float32 resolution of a world position added to the
# pose: the tasks place their envs on a grid hundreds of metres wide, where one ulp of a coordinate is up to
# 3e-5 m (2 ulp = 2.4e-7 relative)
TOL = dict(H.STATE_TOL, pose=(2e-5, 2.4e-7))


def _make(task, monkeypatch):
    from isaacgymenv_amd.isaacgymenvs.tasks.base import vec_task
    monkeypatch.setattr(vec_task, "EXISTING_SIM", None)
    import isaacgymenvs
    torch.manual_seed(42)
    return isaacgymenvs.make(seed=42, task=task, num_envs=N, sim_device="cuda:0", rl_device="cuda:0", headless=True,
                             force_render=False)


def _run_task(env, na, steps=30, seed=7):
    gen = torch.Generator(device="cuda:0").manual_seed(seed)
    for _ in range(steps):
        env.step(2 * torch.rand((N, na), device="cuda:0", generator=gen) - 1)
    torch.cuda.synchronize()
    return gen


def _sim_inputs(env, flat, nd):
    root, dof = H.read_state(env.sim, nd)
    mu = np.ascontiguousarray(env.sim.shape_mu.cpu().numpy().T[:, :flat["ns"]], dtype=np.float64)
    return root, dof, mu


def test_ant_4096_one_simulate_matches_oracle(monkeypatch):
    env = _make("Ant", monkeypatch)
    art, flat = H.ant()
    assert env.sim.kernel_variant == 1 and env.sim.num_sensors == 4
    gen = _run_task(env, 8)
    root, dof, mu = _sim_inputs(env, flat, 8)
    # the task's own torque rule for the next actions (ant.py:281-285)
    act = 2 * torch.rand((N, 8), device="cuda:0", generator=gen) - 1
    tau_t = (act * env.joint_gears * env.power_scale).contiguous()
    tau = tau_t.double().cpu().numpy()
    env.sim.dof_force.copy_(tau_t.reshape(-1))
    env.gym.simulate(env.sim)
    torch.cuda.synchronize()
    g_root, g_dof = H.read_state(env.sim, 8)
    g_sens = env.sim.sens_soa.cpu().numpy().astype(np.float64).T.reshape(N, 4, 6)
    assert np.all(np.isfinite(g_root)) and np.all(np.isfinite(g_dof)) and np.all(np.isfinite(g_sens))
    # the config's physx.solver_type (Ant.yaml asks TGS): the oracle's TGS restatement is its solver_type 3
    ap = dict(H.ANT_PARAMS, solver_type=3 if env.sim.cparams.solver_type == 1 else 0)
    o_root, o_dof, _, o_sens = H.oracle_run(flat, ap, root, dof, tau, mu, nsens=4, sensor_bodies=H.ANT_FEET)
    near_limit = ((dof[:, :, 0] < flat["lower"] + 0.1) | (dof[:, :, 0] > flat["upper"] - 0.1)).any(axis=1)
    assert near_limit.mean() > 0.05, "the sampled states must exercise the joint-limit rows"
    assert np.abs(o_sens).sum() > 0

    def rerun(idx, rng, bits):
        r, d = H.perturbed(root, dof, idx, rng)
        o_r, o_d, _, o_s = H.oracle_run(flat, ap, r, d, tau[idx], mu[idx], bits, nsens=4,
                                        sensor_bodies=H.ANT_FEET)
        return H.state_fields(o_r, o_d, sens=o_s)
    try:
        H.assert_close_or_explained(H.state_fields(g_root, g_dof, sens=g_sens),
                                    H.state_fields(o_root, o_dof, sens=o_sens), rerun, tol=TOL,
                                    what=f"ant {N} envs (30 task steps), one simulate vs oracle")
    except AssertionError:
        H.parity_dump("ant4096", root=root, dof=dof, mu=mu, tau=tau, g_root=g_root, g_dof=g_dof, g_sens=g_sens)
        raise


def test_hound_4096_split_simulate_matches_oracle(monkeypatch):
    env = _make("UsefulHound", monkeypatch)
    art, flat = H.hound()
    assert env.sim.kernel_variant == 1 and env.sim.num_bodies == 24
    _run_task(env, 18)
    root, dof, mu = _sim_inputs(env, flat, 18)
    rng = np.random.RandomState(17)
    tau = np.concatenate([rng.uniform(-80, 80, (N, 12)), rng.uniform(-20, 20, (N, 6))], axis=1)
    env.sim.dof_force.copy_(torch.from_numpy(tau.astype(np.float32).reshape(-1)).cuda())
    env.gym.simulate(env.sim)
    env.gym.refresh_net_contact_force_tensor(env.sim)
    torch.cuda.synchronize()
    g_root, g_dof = H.read_state(env.sim, 18)
    g_cf = env.sim.contact_tensor.cpu().numpy().astype(np.float64).reshape(N, 24, 3)
    assert np.all(np.isfinite(g_root)) and np.all(np.isfinite(g_dof)) and np.all(np.isfinite(g_cf))
    hp = dict(H.HOUND_PARAMS, solver_type=3 if env.sim.cparams.solver_type == 1 else 0)  # UsefulHound.yaml: TGS
    o_root, o_dof, o_cf, _ = H.oracle_run(flat, hp, root, dof, tau, mu, nc=24)
    assert np.abs(o_cf).sum() > 0

    def rerun(idx, rng_, bits):
        r, d = H.perturbed(root, dof, idx, rng_)
        r, d, c, _ = H.oracle_run(flat, hp, r, d, tau[idx], mu[idx], bits, nc=24)
        return H.state_fields(r, d, c)
    try:
        H.assert_close_or_explained(H.state_fields(g_root, g_dof, g_cf), H.state_fields(o_root, o_dof, o_cf), rerun,
                                    tol=TOL, what=f"hound {N} envs (30 task steps), split simulate vs oracle")
    except AssertionError:
        H.parity_dump("hound4096", root=root, dof=dof, mu=mu, tau=tau, g_root=g_root, g_dof=g_dof, g_cf=g_cf)
        raise
