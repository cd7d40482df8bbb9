"""Joint drives (gymapi DOF_MODE_POS / DOF_MODE_VEL with stiffness / damping).

Isaac Gym exposes PhysX articulation joint drives through the dof properties (driveMode, stiffness,
damping) and the target tensors (set_dof_position_target_tensor(_indexed),
set_dof_velocity_target_tensor; the reference's UsefulHound calls the indexed position setter at
useful_hound.py:622-627).  The solver applies them as an implicit spring-damper per substep,
kp (q* - q - h qd) + kd (qd* - qd) with (h kd + h^2 kp) on the mass-matrix diagonal, and a drive whose
force exceeds the dof's effort limit applies the clamped force explicitly; the fp64 oracle restates the
same rule (oracle/physics_oracle.c).  Parity vs PhysX's drive is unpinned (PhysX is
closed and absent).

CPU tests (host backend, no GPU): host vs oracle with random targets (Cartpole, fixed base; Hound,
floating base with ground contacts), a drive holds a pendulum at its target, indexed targets
scatter by actor, per-actor dof properties (drive gains, efforts, velocity and joint limits) against the
oracle run env by env.
GPU tests: the one-env-per-lane kernel vs the oracle, and a drive on ANYmal moves the sim off the
lane-team kernel.
"""
import numpy as np
import pytest
import torch

from oracle.oracle import OracleSim
from tests import helpers as H

DOF_MODE_POS, DOF_MODE_VEL, DOF_MODE_EFFORT = 1, 2, 3


def _cartpole_case(n, seed):
    rng = np.random.RandomState(seed)
    root = np.zeros((n, 13)); root[:, 2] = 2.0; root[:, 6] = 1.0
    dof = np.zeros((n, 2, 2))
    dof[:, :, 0] = 0.4 * (rng.rand(n, 2) - 0.5)
    dof[:, :, 1] = 1.0 * (rng.rand(n, 2) - 0.5)
    tau = np.zeros((n, 2)); tau[:, 0] = rng.uniform(-50, 50, n)
    mu = np.ones((n, 1))
    ptgt = rng.uniform(-0.5, 0.5, (n, 2))
    vtgt = rng.uniform(-0.3, 0.3, (n, 2))
    return root, dof, tau, mu, ptgt, vtgt


CARTPOLE_DRIVES = (np.array([DOF_MODE_POS, DOF_MODE_VEL], dtype=np.int32), np.array([400.0, 0.0]),
                   np.array([30.0, 2.0]))


def _run_sim(kind, n, params, root, dof, tau, mu, ptgt, vtgt, drives, steps, host):
    gym, sim = H.make_gpu_sim(kind, n, params, host=host, drives=drives)
    H.load_state_into(sim, root, dof, mu)
    dev = sim.state.device
    sim.dof_force.copy_(torch.from_numpy(tau.astype(np.float32).reshape(-1)).to(dev))
    from isaacgymenv_amd.isaacgym import gymtorch
    gym.set_dof_position_target_tensor(sim, gymtorch.unwrap_tensor(torch.from_numpy(ptgt.astype(np.float32)).to(dev)))
    gym.set_dof_velocity_target_tensor(sim, gymtorch.unwrap_tensor(torch.from_numpy(vtgt.astype(np.float32)).to(dev)))
    for _ in range(steps):
        gym.simulate(sim)
    if not host:
        torch.cuda.synchronize()
    return gym, sim, H.read_state(sim, dof.shape[1])


def _run_oracle(flat, params, root, dof, tau, mu, ptgt, vtgt, drives, steps, bits=64):
    _, kp, kd = drives
    kp = np.where(drives[0] == DOF_MODE_POS, kp, 0.0)
    kd = np.where((drives[0] == DOF_MODE_POS) | (drives[0] == DOF_MODE_VEL), kd, 0.0)
    r, d, _, _ = H.oracle_run(flat, params, root, dof, tau, mu, bits, steps, drives=(kp, kd), pos_targets=ptgt,
                              vel_targets=vtgt)
    return r, d


def _cartpole_vs_oracle(host):
    n, steps = 64, 20
    art, flat = H.cartpole()
    root, dof, tau, mu, ptgt, vtgt = _cartpole_case(n, seed=7)
    gym, sim, (g_root, g_dof) = _run_sim("cartpole", n, H.CARTPOLE_PARAMS, root, dof, tau, mu, ptgt, vtgt,
                                         CARTPOLE_DRIVES, steps, host)
    o_root, o_dof = _run_oracle(flat, H.CARTPOLE_PARAMS, root, dof, tau, mu, ptgt, vtgt, CARTPOLE_DRIVES, steps)
    np.testing.assert_allclose(g_dof, o_dof, atol=2e-4, rtol=1e-3)
    # the drives are in effect: without them the same 20 steps end elsewhere
    f_root, f_dof = _run_oracle(flat, H.CARTPOLE_PARAMS, root, dof, tau, mu, ptgt, vtgt,
                                (CARTPOLE_DRIVES[0], np.zeros(2), np.zeros(2)), steps)
    assert np.abs(f_dof - o_dof).max() > 1e-2
    return sim


def _hound_vs_oracle(host):
    n = 96
    art, flat = H.hound()
    root, dof, tau, mu = H.hound_states(n, seed=9)
    rng = np.random.RandomState(4)
    mode = np.full(18, DOF_MODE_EFFORT, dtype=np.int32)
    mode[12:] = DOF_MODE_POS  # arm joints position-driven, legs by effort
    kp = np.where(mode == DOF_MODE_POS, 300.0, 7000.0)  # effort dofs keep gains that must be ignored
    kd = np.where(mode == DOF_MODE_POS, 10.0, 50.0)
    drives = (mode, kp, kd)
    ptgt = rng.uniform(-1.0, 1.0, (n, 18))
    vtgt = np.zeros((n, 18))
    gym, sim, (g_root, g_dof) = _run_sim("hound", n, H.HOUND_PARAMS, root, dof, tau, mu, ptgt, vtgt, drives, 1, host)
    o_root, o_dof = _run_oracle(flat, H.HOUND_PARAMS, root, dof, tau, mu, ptgt, vtgt, drives, 1)
    assert np.all(np.isfinite(g_root)) and np.all(np.isfinite(g_dof))

    def rerun(idx, rng, bits):
        r, d = H.perturbed(root, dof, idx, rng)
        return H.state_fields(*_run_oracle(flat, H.HOUND_PARAMS, r, d, tau[idx], mu[idx], ptgt[idx], vtgt[idx],
                                           drives, 1, bits))
    # (Hound's arm-trunk / arm-leg hull contacts switch their support features on fp32 rounding, DESIGN.md 4:
    # 2 of these 96 random states are off, both explained)
    H.assert_close_or_explained(H.state_fields(g_root, g_dof), H.state_fields(o_root, o_dof), rerun,
                                max_env_frac=0.03, what=f"hound arm drives {'host' if host else 'gpu'} vs oracle")
    return sim


def test_cartpole_drives_host_match_oracle():
    _cartpole_vs_oracle(host=True)


def test_hound_arm_drives_host_match_oracle():
    _hound_vs_oracle(host=True)


def test_position_drive_holds_pendulum_at_target():
    """Pole under gravity with a stiff position drive and no actuation settles at its target
    (steady-state error = gravity torque / kp)."""
    n = 8
    drives = (np.array([DOF_MODE_POS, DOF_MODE_POS], dtype=np.int32), np.array([2000.0, 2000.0]),
              np.array([200.0, 200.0]))
    root = np.zeros((n, 13)); root[:, 2] = 2.0; root[:, 6] = 1.0
    dof = np.zeros((n, 2, 2))
    tgt = np.stack([np.linspace(-0.5, 0.5, n), np.linspace(0.4, -0.4, n)], axis=1)
    gym, sim, (g_root, g_dof) = _run_sim("cartpole", n, H.CARTPOLE_PARAMS, root, dof, np.zeros((n, 2)),
                                         np.ones((n, 1)), tgt, np.zeros((n, 2)), drives, 300, True)
    np.testing.assert_allclose(g_dof[:, :, 0], tgt, atol=5e-3)
    assert np.abs(g_dof[:, :, 1]).max() < 1e-2


def test_saturated_drive_is_limited_by_effort():
    """A drive whose force exceeds the dof's effort limit applies the limit (PhysX: the drive's max
    force is the dof's effort property): a stiff position drive on the cart slider toward a far target
    moves the cart exactly as an actuation force equal to the effort does; host backend = oracle."""
    n, steps = 16, 1
    art, flat = H.cartpole()
    root, dof, _, mu, _, _ = _cartpole_case(n, seed=3)
    eff = float(flat["effort"][0])
    drives = (np.array([DOF_MODE_POS, DOF_MODE_EFFORT], dtype=np.int32), np.array([1.0e5, 0.0]),
              np.array([50.0, 0.0]))
    ptgt = np.zeros((n, 2)); ptgt[:, 0] = 5.0          # 1e5 * ~5 m >> effort: saturated every substep
    vtgt = np.zeros((n, 2))
    zero_tau = np.zeros((n, 2))
    gym, sim, (g_root, g_dof) = _run_sim("cartpole", n, H.CARTPOLE_PARAMS, root, dof, zero_tau, mu, ptgt, vtgt,
                                         drives, steps, True)
    o_root, o_dof = _run_oracle(flat, H.CARTPOLE_PARAMS, root, dof, zero_tau, mu, ptgt, vtgt, drives, steps)
    np.testing.assert_allclose(g_dof, o_dof, atol=2e-5, rtol=1e-4)
    tau_eff = np.zeros((n, 2)); tau_eff[:, 0] = eff
    e_root, e_dof = _run_oracle(flat, H.CARTPOLE_PARAMS, root, dof, tau_eff, mu, ptgt, vtgt,
                                (drives[0], np.zeros(2), np.zeros(2)), steps)
    np.testing.assert_allclose(o_dof, e_dof, atol=1e-12, rtol=1e-12)


def test_indexed_targets_scatter_by_actor():
    n = 6
    gym, sim = H.make_host_sim("cartpole", n, H.CARTPOLE_PARAMS, drives=CARTPOLE_DRIVES)
    from isaacgymenv_amd.isaacgym import gymtorch
    src = torch.arange(2 * n, dtype=torch.float32).reshape(n, 2)
    ids = torch.tensor([1, 4], dtype=torch.int32)
    gym.set_dof_position_target_tensor_indexed(sim, gymtorch.unwrap_tensor(src), gymtorch.unwrap_tensor(ids), 2)
    got = sim.pos_target.reshape(n, 2)
    want = torch.zeros(n, 2)
    want[[1, 4]] = src[[1, 4]]
    assert torch.equal(got, want)


def _random_actor_props(gym, sim, rng, modes=(DOF_MODE_POS, DOF_MODE_VEL, DOF_MODE_EFFORT), limit_p=0.5,
                        effort=(20.0, 400.0), kp=(50.0, 600.0), kd=(1.0, 30.0), vel=(2.0, 30.0), lim=(0.05, 0.6)):
    """Every actor its own dof properties (set_actor_dof_properties actor by actor, as anymal_terrain.py:283 /
    useful_hound.py:422 call it): random drive modes, gains, efforts, velocity limits and joint limits.  Returns
    the per-env effective values (kp, kd, effort, lower, upper, has_limits, velocity) [N][nd]."""
    out = {k: [] for k in ("kp", "kd", "effort", "lower", "upper", "has", "vel")}
    for e in sim.envs:
        p = gym.get_actor_dof_properties(e, 0)
        nd = len(p)
        mode = rng.choice(modes, nd).astype(np.int32)
        p["driveMode"] = mode
        p["stiffness"] = rng.uniform(*kp, nd)
        p["damping"] = rng.uniform(*kd, nd)
        p["effort"] = rng.uniform(*effort, nd)
        p["velocity"] = rng.uniform(*vel, nd)
        has = rng.rand(nd) < limit_p
        p["hasLimits"] = has
        p["lower"] = np.where(has, -rng.uniform(*lim, nd), -3.4028235e38)
        p["upper"] = np.where(has, rng.uniform(*lim, nd), 3.4028235e38)
        gym.set_actor_dof_properties(e, 0, p)
        pos, vel_m = mode == DOF_MODE_POS, mode == DOF_MODE_VEL
        out["kp"].append(np.where(pos, p["stiffness"], 0.0).astype(np.float32).astype(np.float64))
        out["kd"].append(np.where(pos | vel_m, p["damping"], 0.0).astype(np.float32).astype(np.float64))
        for k, f in (("effort", "effort"), ("lower", "lower"), ("upper", "upper"), ("vel", "velocity")):
            out[k].append(p[f].astype(np.float32).astype(np.float64))
        out["has"].append(has.astype(np.int32))
    return {k: np.stack(v) for k, v in out.items()}


def _oracle_per_env(flat, params, props, root, dof, tau, mu, ptgt, vtgt, steps=1, bits=64, idx=None):
    """The oracle run env by env, each with its actor's dof properties in the model (effort, velocity limit,
    joint limits) and drive gains."""
    idx = np.arange(root.shape[0]) if idx is None else idx
    rs, ds = [], []
    for k, e in enumerate(idx):
        fe = dict(flat)
        fe["effort"] = props["effort"][e].copy()
        fe["vmax"] = props["vel"][e].copy()
        fe["has_limits"] = props["has"][e].copy()
        fe["lower"] = np.where(props["has"][e] > 0, props["lower"][e], 0.0)
        fe["upper"] = np.where(props["has"][e] > 0, props["upper"][e], 0.0)
        r, d, _, _ = H.oracle_run(fe, params, root[k:k + 1], dof[k:k + 1], tau[k:k + 1], mu[k:k + 1], bits, steps,
                                  drives=(props["kp"][e], props["kd"][e]), pos_targets=ptgt[k:k + 1],
                                  vel_targets=vtgt[k:k + 1])
        rs.append(r)
        ds.append(d)
    return np.concatenate(rs), np.concatenate(ds)


def _per_actor_cartpole(host):
    n, steps = 48, 10
    art, flat = H.cartpole()
    root, dof, tau, mu, ptgt, vtgt = _cartpole_case(n, seed=21)
    gym, sim = H.make_gpu_sim("cartpole", n, H.CARTPOLE_PARAMS, host=host)
    props = _random_actor_props(gym, sim, np.random.RandomState(5))
    gym2, sim, (g_root, g_dof) = _run_sim_on(gym, sim, root, dof, tau, mu, ptgt, vtgt, steps, host)
    assert sim.dof_env_table is not None and (host or sim.kernel_variant == 1)
    o_root, o_dof = _oracle_per_env(flat, H.CARTPOLE_PARAMS, props, root, dof, tau, mu, ptgt, vtgt, steps)
    np.testing.assert_allclose(g_dof, o_dof, atol=2e-4, rtol=1e-3)
    # the per-actor values are in effect: the first actor's values for every env end elsewhere
    same = {k: np.repeat(v[:1], n, axis=0) for k, v in props.items()}
    f_root, f_dof = _oracle_per_env(flat, H.CARTPOLE_PARAMS, same, root, dof, tau, mu, ptgt, vtgt, steps)
    assert np.abs(f_dof - o_dof).max() > 1e-2


def _run_sim_on(gym, sim, root, dof, tau, mu, ptgt, vtgt, steps, host):
    H.load_state_into(sim, root, dof, mu)
    dev = sim.state.device
    sim.dof_force.copy_(torch.from_numpy(tau.astype(np.float32).reshape(-1)).to(dev))
    from isaacgymenv_amd.isaacgym import gymtorch
    gym.set_dof_position_target_tensor(sim, gymtorch.unwrap_tensor(torch.from_numpy(ptgt.astype(np.float32)).to(dev)))
    gym.set_dof_velocity_target_tensor(sim, gymtorch.unwrap_tensor(torch.from_numpy(vtgt.astype(np.float32)).to(dev)))
    for _ in range(steps):
        gym.simulate(sim)
    if not host:
        torch.cuda.synchronize()
    return gym, sim, H.read_state(sim, dof.shape[1])


def _per_actor_anymal(host):
    """Floating base with ground contacts: ANYmal, every actor its own drive gains, efforts, velocity and joint
    limits (the one-env-per-lane kernel / the host backend) against the oracle env by env."""
    n = 64
    art, flat = H.anymal()
    root, dof, tau, mu = H.anymal_states(n, seed=12)
    rng = np.random.RandomState(8)
    gym, sim = H.make_gpu_sim("anymal", n, H.ANYMAL_PARAMS, host=host)
    props = _random_actor_props(gym, sim, rng, effort=(30.0, 120.0), kp=(20.0, 200.0), kd=(0.5, 6.0))
    ptgt = dof[:, :, 0] + rng.uniform(-0.3, 0.3, (n, 12))
    vtgt = rng.uniform(-1.0, 1.0, (n, 12))
    gym, sim, (g_root, g_dof) = _run_sim_on(gym, sim, root, dof, tau, mu, ptgt, vtgt, 1, host)
    assert host or sim.kernel_variant == 1
    o_root, o_dof = _oracle_per_env(flat, H.ANYMAL_PARAMS, props, root, dof, tau, mu, ptgt, vtgt)

    def rerun(idx, rng_, bits):
        r, d = H.perturbed(root, dof, idx, rng_)
        return H.state_fields(*_oracle_per_env(flat, H.ANYMAL_PARAMS, props, r, d, tau[idx], mu[idx], ptgt[idx],
                                               vtgt[idx], 1, bits, idx=idx))
    H.assert_close_or_explained(H.state_fields(g_root, g_dof), H.state_fields(o_root, o_dof), rerun,
                                max_env_frac=0.05, what=f"anymal per-actor dof properties {'host' if host else 'gpu'} "
                                                        f"vs oracle")


def test_per_actor_dof_properties_host_match_oracle():
    """actors with differing drive gains, efforts and limits are no longer refused; the host
    backend reads them from the per-actor table (gymsim.h gs_sim_bind_dof_properties_env) and matches the oracle
    run env by env with each actor's values."""
    _per_actor_cartpole(host=True)


def test_per_actor_dof_properties_anymal_host_match_oracle():
    _per_actor_anymal(host=True)


@pytest.mark.gpu
def test_per_actor_dof_properties_gpu_match_oracle():
    _per_actor_cartpole(host=False)


@pytest.mark.gpu
def test_per_actor_dof_properties_anymal_gpu_match_oracle():
    _per_actor_anymal(host=False)


def test_uniform_dof_properties_keep_the_asset_path():
    """Actors with the same properties as the asset bind no table (the lane-team kernel stays selectable)."""
    gym, sim = H.make_host_sim("cartpole", 3, H.CARTPOLE_PARAMS, drives=CARTPOLE_DRIVES)
    gym.simulate(sim)
    assert sim.dof_env_table is None
    props = gym.get_actor_dof_properties(sim.envs[2], 0)
    props["effort"][1] = 7.0
    gym.set_actor_dof_properties(sim.envs[2], 0, props)
    gym.simulate(sim)
    assert sim.dof_env_table is not None and float(sim.dof_env_table[2, 1, 2]) == 7.0


def test_gains_of_undriven_dofs_may_differ_between_actors():
    """Only effective gains count (stiffness where driveMode is POS, damping where POS or VEL): actors whose
    EFFORT dofs carry different stiffness / damping values are accepted."""
    gym, sim = H.make_host_sim("cartpole", 2, H.CARTPOLE_PARAMS)
    for i, e in enumerate(sim.envs):
        props = gym.get_actor_dof_properties(e, 0)
        props["driveMode"][:] = DOF_MODE_EFFORT
        props["stiffness"][:] = 10.0 * (i + 1)
        props["damping"][:] = 3.0 * (i + 1)
        gym.set_actor_dof_properties(e, 0, props)
    gym.simulate(sim)
    assert not sim.drives_dirty


def test_drives_updated_after_prepare_take_effect():
    """Dof properties set actor by actor after prepare_sim are uploaded before the next simulate."""
    n = 4
    gym, sim = H.make_host_sim("cartpole", n, H.CARTPOLE_PARAMS)
    for e in sim.envs:
        props = gym.get_actor_dof_properties(e, 0)
        props["driveMode"], props["stiffness"], props["damping"] = CARTPOLE_DRIVES
        gym.set_actor_dof_properties(e, 0, props)
    gym.simulate(sim)
    assert not sim.drives_dirty


@pytest.mark.gpu
def test_cartpole_drives_gpu_match_oracle():
    sim = _cartpole_vs_oracle(host=False)
    assert sim.kernel_variant == 1


@pytest.mark.gpu
def test_hound_arm_drives_gpu_match_oracle():
    _hound_vs_oracle(host=False)


@pytest.mark.gpu
def test_anymal_drives_leave_the_lane_team_kernel():
    """ANYmal runs the lane-team kernel, which has no drive terms; position drives select the
    one-env-per-lane kernel, and its step matches the oracle."""
    n = 128
    art, flat = H.anymal()
    gym, sim = H.make_gpu_sim("anymal", n, H.ANYMAL_PARAMS)
    assert sim.kernel_variant == 2
    root, dof, tau, mu = H.anymal_states(n, seed=2)
    mode = np.full(12, DOF_MODE_POS, dtype=np.int32)
    drives = (mode, np.full(12, 80.0), np.full(12, 2.0))
    ptgt = np.tile(dof[:, :, 0].mean(0), (n, 1)) + 0.1
    gym, sim, (g_root, g_dof) = _run_sim("anymal", n, H.ANYMAL_PARAMS, root, dof, tau, mu, ptgt,
                                         np.zeros((n, 12)), drives, 1, False)
    assert sim.kernel_variant == 1
    o_root, o_dof = _run_oracle(flat, H.ANYMAL_PARAMS, root, dof, tau, mu, ptgt, np.zeros((n, 12)), drives, 1)
    def rerun(idx, rng, bits):
        r, d = H.perturbed(root, dof, idx, rng)
        return H.state_fields(*_run_oracle(flat, H.ANYMAL_PARAMS, r, d, tau[idx], mu[idx], ptgt[idx],
                                           np.zeros((len(idx), 12)), drives, 1, bits))
    H.assert_close_or_explained(H.state_fields(g_root, g_dof), H.state_fields(o_root, o_dof), rerun,
                                max_env_frac=5e-3, what="anymal drives gpu (one env per lane) vs oracle")
