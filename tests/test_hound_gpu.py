"""UsefulHound row on the GPU: the HIP kernels against the fp64 oracles.

* link kinematics (gs_kinematics.hip) vs oracle/kinematics_oracle.py -- rigid-body state,
  Jacobian and mass matrix for Hound (24 links welded into 19 bodies), ANYmal and Cartpole;
  fp32 vs fp64 tolerances: positions / Jacobian entries 2e-5 + 1e-5 relative, velocities 1e-4
  + 1e-4 relative, mass matrix 1e-4 + 1e-4 relative, quaternions |q . q_oracle| >= 1 - 1e-6;
* physics (Topo_hound, one env per lane, 84 plane-contact candidates, joint limits) vs
  oracle/physics_oracle.c -- the ANYmal tolerances of DESIGN.md section 4, contact forces per
  reported link (the foot sphere reports at the foot link, not at the calf it is welded to);
* the task on the real simulator: a standing episode, OSC arm torques finite and clamped.
"""
import numpy as np
import pytest
import torch

from oracle import kinematics_oracle as KO
from oracle.oracle import OracleSim
from tests import helpers as H

pytestmark = pytest.mark.gpu


def _kin_case(kind, n, seed):
    if kind == "hound":
        art, flat = H.hound()
        root, dof, _, mu = H.hound_states(n, seed=seed)
        params = H.HOUND_PARAMS
    elif kind == "anymal":
        art, flat = H.anymal()
        root, dof, _, mu = H.anymal_states(n, seed=seed)
        params = H.ANYMAL_PARAMS
    else:
        art, flat = H.cartpole()
        rng = np.random.RandomState(seed)
        root = np.zeros((n, 13)); root[:, 2] = 2.0; root[:, 6] = 1.0
        dof = rng.uniform(-1.5, 1.5, (n, 2, 2))
        mu = np.ones((n, flat["ns"]))
        params = H.CARTPOLE_PARAMS
    return art, flat, root, dof, mu, params


@pytest.mark.parametrize("kind", ["hound", "anymal", "cartpole"])
def test_link_kinematics_match_oracle(kind):
    n = 300
    art, flat, root, dof, mu, params = _kin_case(kind, n, seed=21)
    gym, sim = H.make_gpu_sim(kind, n, params)
    # root pose of the cartpole is fixed by the sim (the rail sits at its start pose)
    if kind == "cartpole":
        root = np.zeros((n, 13)); root[:, 2] = 2.0; root[:, 6] = 1.0
    H.load_state_into(sim, root, dof, mu)
    from isaacgymenv_amd.isaacgym import gymtorch
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    jac_t = gymtorch.wrap_tensor(gym.acquire_jacobian_tensor(sim, kind))
    mm_t = gymtorch.wrap_tensor(gym.acquire_mass_matrix_tensor(sim, kind))
    gym.refresh_rigid_body_state_tensor(sim)
    gym.refresh_jacobian_tensors(sim)
    gym.refresh_mass_matrix_tensors(sim)
    torch.cuda.synchronize()
    o_rb, o_jac, o_mm = KO.batch(flat, root, dof)
    g_rb = rb.cpu().numpy().astype(np.float64)
    nr, nv = flat["nr"], flat["nd"] + (0 if flat["fixed_base"] else 6)
    assert g_rb.shape == (n * nr, 13) and tuple(mm_t.shape) == (n, nv, nv)
    if flat["fixed_base"]:
        assert tuple(jac_t.shape) == (n, nr - 1, 6, nv)  # Isaac Gym drops the welded root row
        g_jac = np.concatenate([np.zeros((n, 1, 6, nv)), jac_t.cpu().numpy()], axis=1)
    else:
        assert tuple(jac_t.shape) == (n, nr, 6, nv)
        g_jac = jac_t.cpu().numpy().astype(np.float64)
    np.testing.assert_allclose(g_rb[:, 0:3], o_rb[:, 0:3], atol=2e-5, rtol=1e-5)
    dots = np.abs(np.sum(g_rb[:, 3:7] * o_rb[:, 3:7], axis=1))
    assert dots.min() >= 1 - 1e-6, dots.min()
    np.testing.assert_allclose(g_rb[:, 7:13], o_rb[:, 7:13], atol=1e-4, rtol=1e-4)
    np.testing.assert_allclose(g_jac, o_jac, atol=2e-5, rtol=1e-5)
    np.testing.assert_allclose(mm_t.cpu().numpy(), o_mm, atol=1e-4, rtol=1e-4)


def _hound_gpu(n, root, dof, tau, mu, steps=1):
    gym, sim = H.make_gpu_sim("hound", n, H.HOUND_PARAMS)
    assert sim.kernel_variant == 1 and sim.num_bodies == 24
    H.load_state_into(sim, root, dof, mu)
    for _ in range(steps):
        sim.dof_force.copy_(torch.from_numpy(tau.astype(np.float32).reshape(-1)))
        gym.simulate(sim)
    gym.refresh_net_contact_force_tensor(sim)
    torch.cuda.synchronize()
    g_root, g_dof = H.read_state(sim, 18)
    g_cf = sim.contact_tensor.cpu().numpy().astype(np.float64).reshape(n, 24, 3)
    return g_root, g_dof, g_cf


def test_hound_one_simulate_matches_oracle():
    n = 256
    art, flat = H.hound()
    root, dof, tau, mu = H.hound_states(n, seed=5)
    g_root, g_dof, g_cf = _hound_gpu(n, root, dof, tau, mu)
    osim = OracleSim(flat, H.HOUND_PARAMS)
    o_root, o_dof = root.copy(), dof.copy()
    o_cf = np.zeros((n, 24, 3))
    osim.simulate(o_root, o_dof, np.ascontiguousarray(tau), mu, o_cf)
    assert np.all(np.isfinite(g_root)) and np.all(np.isfinite(g_dof))
    assert np.abs(o_cf).sum() > 0, "some feet / boxes must be in contact in the sampled states"
    def rerun(idx, rng, bits):
        r, d = H.perturbed(root, dof, idx, rng)
        r, d, c, _ = H.oracle_run(flat, H.HOUND_PARAMS, r, d, tau[idx], mu[idx], bits, nc=24)
        return H.state_fields(r, d, c)
    H.assert_close_or_explained(H.state_fields(g_root, g_dof, g_cf), H.state_fields(o_root, o_dof, o_cf), rerun,
                                what="hound gpu")
    # the foot spheres report at the foot links, never at the calves they are welded to
    names = art.link_names()
    feet = [names.index(f"{l}_foot") for l in ("FL", "FR", "RL", "RR")]
    assert np.abs(o_cf[:, feet]).sum() > 0


def test_hound_standing_rollout_tracks_oracle():
    """PD standing (legs at the task's default angles) for 30 env steps x 5 simulates."""
    n = 64
    art, flat = H.hound()
    q0 = np.array([0.0, 0.7854, -1.5708] * 4 + [0.0] * 6)
    root = np.zeros((n, 13)); root[:, 2] = 0.62; root[:, 6] = 1.0
    dof = np.zeros((n, 18, 2)); dof[:, :, 0] = q0
    mu = np.ones((n, flat["ns"]))
    gym, sim = H.make_gpu_sim("hound", n, H.HOUND_PARAMS)
    H.load_state_into(sim, root, dof, mu)
    osim = OracleSim(flat, H.HOUND_PARAMS)
    r, d = root.copy(), dof.copy()
    # arm unactuated: a PD on its light distal links (end_link 0.019 kg) is explicit-damping unstable
    # at h = 5 ms and chatters on its velocity limits, which fp32 / fp64 do not track alike
    kp = np.array([80.0] * 12 + [0.0] * 6)
    kd = np.array([2.0] * 12 + [0.0] * 6)
    for _ in range(30 * 5):
        tau = np.clip(kp * (q0 - d[:, :, 0]) - kd * d[:, :, 1], -80, 80)
        g_root, g_dof = H.read_state(sim, 18)
        g_tau = np.clip(kp * (q0 - g_dof[:, :, 0]) - kd * g_dof[:, :, 1], -80, 80)
        sim.dof_force.copy_(torch.from_numpy(g_tau.astype(np.float32).reshape(-1)))
        gym.simulate(sim)
        osim.simulate(r, d, np.ascontiguousarray(tau), mu)
    torch.cuda.synchronize()
    g_root, g_dof = H.read_state(sim, 18)
    np.testing.assert_allclose(g_root[:, 0:3], r[:, 0:3], atol=1e-3)
    np.testing.assert_allclose(g_dof[:, :12, 0], d[:, :12, 0], atol=1e-3)
    np.testing.assert_allclose(g_dof[:, 12:, 0], d[:, 12:, 0], atol=1e-2)
    assert 0.3 < g_root[:, 2].mean() < 0.62  # on its feet


def _make(n, monkeypatch, **over):
    from isaacgymenv_amd.isaacgymenvs.tasks.base import vec_task
    monkeypatch.setattr(vec_task, "EXISTING_SIM", None)
    import isaacgymenvs
    torch.manual_seed(42)
    ov = [f"{k}={v}" for k, v in over.items()]
    return isaacgymenvs.make(seed=42, task="UsefulHound", num_envs=n, sim_device="cuda:0", rl_device="cuda:0",
                             headless=True, force_render=False, overrides=ov)


def test_hound_task_episode(monkeypatch):
    """The task on the real simulator: zero actions hold the legs at their default angles and the
    arm under OSC; the robots stand, observations stay finite, arm torques stay within limits;
    random actions run a full episode length with resets."""
    n = 256
    env = _make(n, monkeypatch)
    assert env.obs_buf.shape == (n, 204) and env.num_actions == 18
    assert env.contact_forces.shape == (n, 24, 3)
    assert env._j_eef.shape == (n, 6, 6) and env._mm.shape == (n, 6, 6)
    zero = torch.zeros((n, 18), device="cuda:0")
    env.step(zero)
    for _ in range(60):
        obs, rew, reset, extras = env.step(zero)
    assert torch.isfinite(obs["obs"]).all() and torch.isfinite(rew).all()
    z = env.root_states[:, 2]
    assert 0.3 < float(z.median()) < 0.7, float(z.median())
    assert float(env.torques[:, 12:].abs().max()) <= float(env._houndarm_effort_limits.max()) + 1e-3
    feet_fz = env.contact_forces[:, env.feet_indices, 2]
    assert float((feet_fz > 1.0).float().mean()) > 0.5, "standing robots carry their weight on the feet"
    gen = torch.Generator(device="cuda:0").manual_seed(3)
    resets = 0
    for t in range(300):
        a = 2 * torch.rand((n, 18), device="cuda:0", generator=gen) - 1
        obs, rew, reset, extras = env.step(a)
        resets += int(reset.sum())
        if t % 50 == 0:
            assert torch.isfinite(obs["obs"]).all() and torch.isfinite(rew).all()
    assert resets > 0


def _osc_reference_f64(J, M, v_eef, q, qd, dpose, kp, kd, kp_null, kd_null, default, effort):
    """useful_hound.py:660-691 in float64 numpy (the oracle of gt_hound_control's arm half)."""
    mm_inv = np.linalg.inv(M)
    m_eef = np.linalg.inv(J @ mm_inv @ np.transpose(J, (0, 2, 1)))
    u = np.transpose(J, (0, 2, 1)) @ m_eef @ (kp * dpose - kd * v_eef)[..., None]
    j_eef_inv = m_eef @ J @ mm_inv
    u_null = kd_null * -qd + kp_null * (np.mod(default - q + np.pi, 2 * np.pi) - np.pi)
    u_null = M @ u_null[..., None]
    u = u + (np.eye(6)[None] - np.transpose(J, (0, 2, 1)) @ j_eef_inv) @ u_null
    return np.clip(u[..., 0], -effort, effort)


def test_hound_control_kernel_matches_reference(monkeypatch):
    """gt_hound_control (legs PD + arm OSC, one kernel) vs the reference expressions: the legs against
    torch float32 on the same tensors (same expression order), the arm against float64 numpy."""
    n = 512
    env = _make(n, monkeypatch)
    gen = torch.Generator(device="cuda:0").manual_seed(11)
    for _ in range(20):
        env.step(2 * torch.rand((n, 18), device="cuda:0", generator=gen) - 1)
    torch.cuda.synchronize()
    a = (2 * torch.rand((n, 18), device="cuda:0", generator=gen) - 1).contiguous()
    out = torch.zeros((n, 18), device="cuda:0")
    env._control(a, out)
    torch.cuda.synchronize()
    legs = torch.clip(env.Kp * (env.action_scale * a[:, :12] + env.hound_default_dof_pos - env.hound_dof_pos)
                      - env.Kd * env.hound_dof_vel, -80.0, 80.0)
    torch.testing.assert_close(out[:, :12], legs, rtol=0, atol=1e-5)
    f = lambda t: t.detach().double().cpu().numpy()  # noqa: E731
    dpose = f(a[:, 12:] * env.arm_cmd_limit / env.arm_action_scale)
    ref = _osc_reference_f64(f(env._j_eef), f(env._mm), f(env._eef_state[:, 7:]), f(env._q[:, :6]), f(env._qd[:, :6]),
                             dpose, f(env.arm_kp), f(env.arm_kd), f(env.arm_kp_null), f(env.arm_kd_null),
                             f(env.houndarm_default_dof_pos[:6]), f(env._houndarm_effort_limits[:6]))
    got = f(out[:, 12:])
    scale = np.maximum(1.0, np.abs(ref))
    assert np.all(np.abs(got - ref) <= 1e-4 * scale), np.abs(got - ref).max()
    np.testing.assert_array_equal(f(env._effort_control[:, :6]), got)


def _pd_sequence(flat, params, root, dof, dof_tensor, mu, act, default, kp, kd, scale, decimation, extra, bits=64):
    """anymal_terrain.py:443-451's decimation loop (+ the extra simulate) on the oracle: the first PD torque from
    the stale dof tensor, the next from the oracle's own state (the same sequence gs_sim_pd_step fuses)."""
    dt = np.float64 if bits == 64 else np.float32
    c = lambda a: np.array(a, dtype=dt, order="C")  # a copy: the oracle steps it in place  # noqa: E731
    sim = OracleSim(flat, params, real_bits=bits)
    r, d, mu = c(root), c(dof), c(mu)
    cf = np.zeros((root.shape[0], flat["nr"], 3), dt)
    q, qd = dof_tensor[:, :, 0], dof_tensor[:, :, 1]
    tau = None
    for i in range(decimation + extra):
        if i < decimation:
            tau = np.clip(kp * (scale * act + default - q) - kd * qd, -80.0, 80.0)
        sim.simulate(r, d, c(tau), mu, cf)
        q, qd = d[:, :, 0].copy(), d[:, :, 1].copy()
    f = lambda a: np.asarray(a, np.float64)  # noqa: E731
    return dict(q=f(d[:, :, 0]), qd=f(d[:, :, 1]), pose=f(r[:, :7]), vel=f(r[:, 7:]), tau=f(tau), cf=f(cf))


def _hound_pd_case(root, dof, mu, act, decimation, extra):
    n = root.shape[0]
    gym, sim = H.make_gpu_sim("hound", n, H.HOUND_PARAMS)
    H.load_state_into(sim, root, dof, mu)
    gym.refresh_dof_state_tensor(sim)
    torch.cuda.synchronize()
    dof_tensor = sim.dof_tensor.view(n, 18, 2).double().cpu().numpy()
    default = np.array([0.0, 0.7854, -1.5708] * 4 + [0.0] * 6)
    kp, kd, scale = 80.0, 2.0, 0.5
    torques = torch.empty((n, 18), device="cuda:0")
    gym.amd_pd_decimation_step(sim, torch.from_numpy(act.astype(np.float32)).cuda(),
                               torch.from_numpy(default.astype(np.float32)).cuda(), kp, kd, scale, 80.0, decimation,
                               extra, torques)
    torch.cuda.synchronize()
    g_root, g_dof = H.read_state(sim, 18)
    gpu = dict(q=g_dof[:, :, 0], qd=g_dof[:, :, 1], pose=g_root[:, :7], vel=g_root[:, 7:],
               tau=torques.double().cpu().numpy(), cf=sim.contact_tensor.double().cpu().numpy().reshape(n, 24, 3))
    args = (dof_tensor, act, default, kp, kd, scale, decimation, extra)
    return gpu, args


# tolerances of the 4 x PD + 1 sequence (5 substeps; test_headline_oracle_gpu.py)
SEQ_TOL = {"q": (1e-4, 0.0), "qd": (2.5e-2, 2.5e-2), "pose": (1e-4, 0.0), "vel": (2.5e-2, 2.5e-2), "tau": (0.5, 1e-2),
           "cf": (2.0, 5e-2)}


def test_hound_fused_pd_step_with_self_collision_matches_oracle():
    """gs_sim_pd_step on UsefulHound's topology runs the wave-assisted PD kernel (k_pd_step_wave: the
    near-pair records in the env columns), a different narrowphase route than its simulate (the split
    records kernel) -- ADVICE r03: this combination had no GPU test.  From random states (arm on the trunk,
    legs and arm moving) against the oracle, every env within tolerance or explained: (1) one PD evaluation +
    one substep; (2) the full 4 x decimation + 1 sequence (the r04f failure of this case, env 111,
    was the float GJK stalling on a cylinder rim plus a checker that perturbed the stepped state, DESIGN.md
    3.12); (3) the 4 x PD + 1 sequence from the standing pose, where nothing is chaotic, to the one-simulate
    bounds."""
    n = 256
    art, flat = H.hound()
    root, dof, tau, mu = H.hound_states(n, seed=13, spread=0.5)
    act = np.random.RandomState(2).uniform(-1.0, 1.0, (n, 18))
    for decimation, extra, tol in ((1, 0, dict(H.STATE_TOL, tau=(0.5, 1e-2))), (4, 1, SEQ_TOL)):
        gpu, args = _hound_pd_case(root, dof, mu, act, decimation, extra)
        ref = _pd_sequence(flat, H.HOUND_PARAMS, root, dof, args[0], mu, *args[1:])
        assert np.abs(ref["cf"]).sum() > 0

        def rerun(idx, rng_, bits):
            r, d = H.perturbed(root, dof, idx, rng_)
            return _pd_sequence(flat, H.HOUND_PARAMS, r, d, args[0][idx], mu[idx], act[idx], *args[2:], bits)
        H.assert_close_or_explained(gpu, ref, rerun, tol=tol, max_env_frac=0.03,
                                    what=f"hound fused pd step (wave-assisted self-collision), {decimation} x PD + "
                                         f"{extra}, vs oracle")
    # standing: the task's start pose (useful_hound.py default angles), small random actions, 4 x PD + 1
    q0 = np.array([0.0, 0.7854, -1.5708] * 4 + [0.0] * 6)
    root = np.zeros((n, 13)); root[:, 0] = np.arange(n) * 2.0; root[:, 2] = 0.62; root[:, 6] = 1.0
    dof = np.zeros((n, 18, 2)); dof[:, :, 0] = q0
    mu = np.ones((n, flat["ns"]))
    act = 0.2 * np.random.RandomState(3).uniform(-1.0, 1.0, (n, 18))
    gpu, args = _hound_pd_case(root, dof, mu, act, 4, 1)
    ref = _pd_sequence(flat, H.HOUND_PARAMS, root, dof, args[0], mu, *args[1:])
    for k, (at, rt) in dict(q=(1e-4, 0.0), pose=(1e-4, 0.0), qd=(2.5e-2, 2.5e-2), vel=(2.5e-2, 2.5e-2),
                            tau=(0.5, 1e-2)).items():
        np.testing.assert_allclose(gpu[k], ref[k], atol=at, rtol=rt, err_msg=k)
