"""The product's CPU pipeline (sim_device=cpu pipeline=cpu; BASELINE config 1) without a GPU.

libgymsim's host backend (gs_host.hip) runs the same solver source as the HIP kernels
(gs_solver.h / gs_kinematics.h are __host__ __device__) on a thread pool, on host tensors.
Reference: vec_task.py:82-88 (device selection), cfg/config.yaml:30-32 (physx.num_threads 4),
cfg/task/Cartpole.yaml:27-32 (use_gpu_pipeline / physx.use_gpu from pipeline / sim_device).

Checked here, on CPU only (these are `-m "not gpu"` tests):
  * one simulate from identical states vs the fp64 oracle with the GPU tests' tolerances
    (DESIGN.md section 4): Cartpole, ANYmal (plane), Ant (limits + force sensors), Hound
    (per-link contact forces), ANYmal on a rough trimesh; link kinematics vs the kinematics oracle;
  * the thread count does not change a single bit (one env per task, no cross-env reduction);
  * the fused decimation step equals the unfused gym call sequence on the host backend too;
  * Cartpole 64 through isaacgymenvs.make(sim_device="cpu", pipeline=cpu): every env step of the
    real sim tracks an oracle step from the same state, resets / timeouts behave as the reference's,
    and the reward / done function reproduces tests/golden/cartpole.npz (reference outputs) on the
    fixture's own observations (dynamics free).
"""
import os

import numpy as np
import pytest
import torch

from oracle import kinematics_oracle as KO
from oracle.oracle import OracleSim
from tests import helpers as H

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _oracle(flat, params, root, dof, tau, mu, steps=1, **kw):
    sim = OracleSim(flat, params, **{k: v for k, v in kw.items() if k in ("sensor_bodies", "terrain")})
    r, d = root.copy(), dof.copy()
    cf = np.zeros((root.shape[0], flat["nr"], 3))
    sens = kw.get("sens")
    for _ in range(steps):
        if sens is not None:
            sim.simulate(r, d, np.ascontiguousarray(tau), mu, cf, sens=sens)
        else:
            sim.simulate(r, d, np.ascontiguousarray(tau), mu, cf)
    return r, d, cf


def _host(kind, n, params, root, dof, tau, mu, nd, steps=1, terrain=None, threads=4):
    gym, sim = H.make_host_sim(kind, n, params, terrain=terrain, threads=threads)
    assert sim.host and sim.kernel_variant == 3 and sim.state.device.type == "cpu"
    H.load_state_into(sim, root, dof, mu)
    sim.dof_force.copy_(torch.from_numpy(tau.astype(np.float32).reshape(-1)))
    for _ in range(steps):
        gym.simulate(sim)
    g_root, g_dof = H.read_state(sim, nd)
    return gym, sim, g_root, g_dof


def _explained(g, o, flat, params, root, dof, tau, mu, what, **kw):
    """Host results vs the oracle: every env within the GPU bars or its difference the oracle's own
    sensitivity (H.assert_close_or_explained)."""
    def rerun(idx, rng, bits):
        r, d = H.perturbed(root, dof, idx, rng)
        kw2 = {k: v for k, v in kw.items() if k in ("sensor_bodies", "terrain")}
        nsens = kw["sens"].shape[1] if "sens" in kw else 0
        o_r, o_d, o_c, o_s = H.oracle_run(flat, params, r, d, tau[idx], mu[idx], bits, nc=flat["nr"], nsens=nsens,
                                          **kw2)
        return H.state_fields(o_r, o_d, o_c if "cf" in g else None, o_s if "sens" in g else None)
    H.assert_close_or_explained(g, o, rerun, what=what)


def _check_state(g_root, g_dof, o_root, o_dof):
    assert np.all(np.isfinite(g_root)) and np.all(np.isfinite(g_dof))
    np.testing.assert_allclose(g_root[:, 0:7], o_root[:, 0:7], atol=2e-5, rtol=0, err_msg="root pose")
    np.testing.assert_allclose(g_dof[:, :, 0], o_dof[:, :, 0], atol=2e-5, rtol=0, err_msg="dof pos")
    np.testing.assert_allclose(g_root[:, 7:13], o_root[:, 7:13], atol=5e-3, rtol=5e-3, err_msg="root vel")
    np.testing.assert_allclose(g_dof[:, :, 1], o_dof[:, :, 1], atol=5e-3, rtol=5e-3, err_msg="dof vel")


def test_no_gpu_is_used():
    """These tests run on the host backend whether or not a GPU exists (the driver runs them here)."""
    gym, sim = H.make_host_sim("cartpole", 4, H.CARTPOLE_PARAMS)
    assert sim.host and sim.stream() is None
    for t in (sim.state, sim.root_tensor, sim.dof_tensor, sim.contact_tensor):
        assert t.device.type == "cpu"


def test_cartpole_one_simulate_matches_oracle():
    n = 64
    art, flat = H.cartpole()
    rng = np.random.RandomState(3)
    root = np.zeros((n, 13)); root[:, 2] = 2.0; root[:, 6] = 1.0
    dof = np.zeros((n, 2, 2))
    dof[:, :, 0] = 0.2 * (rng.rand(n, 2) - 0.5)
    dof[:, :, 1] = 0.5 * (rng.rand(n, 2) - 0.5)
    tau = np.zeros((n, 2)); tau[:, 0] = rng.uniform(-400, 400, n)
    mu = np.ones((n, flat["ns"]))
    _, _, g_root, g_dof = _host("cartpole", n, H.CARTPOLE_PARAMS, root, dof, tau, mu, 2)
    o_root, o_dof, _ = _oracle(flat, H.CARTPOLE_PARAMS, root, dof, tau, mu)
    np.testing.assert_allclose(g_dof, o_dof, atol=1e-4, rtol=1e-4)


def test_anymal_one_simulate_matches_oracle():
    n = 128
    art, flat = H.anymal()
    root, dof, tau, mu = H.anymal_states(n, seed=1)
    gym, sim, g_root, g_dof = _host("anymal", n, H.ANYMAL_PARAMS, root, dof, tau, mu, 12)
    o_root, o_dof, o_cf = _oracle(flat, H.ANYMAL_PARAMS, root, dof, tau, mu)
    _check_state(g_root, g_dof, o_root, o_dof)
    g_cf = sim.cf_soa.numpy().T.reshape(n, 13, 3)
    np.testing.assert_allclose(g_cf, o_cf, atol=1.0, rtol=2e-2)
    gym.refresh_net_contact_force_tensor(sim)
    np.testing.assert_array_equal(sim.contact_tensor.numpy().reshape(n, 13, 3), g_cf)


def test_ant_limits_and_sensors_match_oracle():
    n = 128
    art, flat = H.ant()
    root, dof, tau, mu = H.ant_states(n, seed=3)
    gym, sim, g_root, g_dof = _host("ant", n, H.ANT_PARAMS, root, dof, tau, mu, 8)
    assert sim.num_sensors == 4
    g_sens = sim.sens_soa.numpy().astype(np.float64).T.reshape(n, 4, 6)
    gym.refresh_force_sensor_tensor(sim)
    np.testing.assert_array_equal(sim.sensor_tensor.numpy().reshape(n, 4, 6), g_sens.astype(np.float32))
    sens = np.zeros((n, 4, 6))
    o_root, o_dof, _ = _oracle(flat, H.ANT_PARAMS, root, dof, tau, mu, sensor_bodies=H.ANT_FEET, sens=sens)
    _explained(H.state_fields(g_root, g_dof, sens=g_sens), H.state_fields(o_root, o_dof, sens=sens), flat, H.ANT_PARAMS,
               root, dof, tau, mu, "ant host", sensor_bodies=H.ANT_FEET, sens=sens)


def test_hound_per_link_contacts_match_oracle():
    n = 96
    art, flat = H.hound()
    root, dof, tau, mu = H.hound_states(n, seed=5)
    gym, sim, g_root, g_dof = _host("hound", n, H.HOUND_PARAMS, root, dof, tau, mu, 18)
    gym.refresh_net_contact_force_tensor(sim)
    g_cf = sim.contact_tensor.numpy().astype(np.float64).reshape(n, 24, 3)
    o_root, o_dof, o_cf = _oracle(flat, H.HOUND_PARAMS, root, dof, tau, mu)
    assert np.abs(o_cf).sum() > 0
    _explained(H.state_fields(g_root, g_dof, g_cf), H.state_fields(o_root, o_dof, o_cf), flat, H.HOUND_PARAMS, root,
               dof, tau, mu, "hound host")


def test_rough_trimesh_matches_oracle():
    ter = H.rough_terrain(seed=5, rows=80, cols=80)
    n = 96
    art, flat = H.anymal()
    params = dict(H.ANYMAL_PARAMS, has_ground=0)
    root, dof, tau, mu = H.anymal_states(n, seed=2)
    rng = np.random.RandomState(102)
    root[:, 0] = rng.uniform(-3.0, 3.0, n)
    root[:, 1] = rng.uniform(-3.0, 3.0, n)
    v = ter["oracle"]["vertices"].reshape(-1, 3)
    for i in range(n):
        near = (np.abs(v[:, 0] - root[i, 0]) < 0.15) & (np.abs(v[:, 1] - root[i, 1]) < 0.15)
        root[i, 2] += v[near, 2].mean() + 0.05
    gym, sim, g_root, g_dof = _host("anymal", n, params, root, dof, tau, mu, 12, terrain=ter)
    o_root, o_dof, o_cf = _oracle(flat, params, root, dof, tau, mu, terrain=ter["oracle"])
    assert np.abs(o_cf).sum(axis=(1, 2)).astype(bool).mean() > 0.5, "most envs must touch the mesh"
    g_cf = sim.cf_soa.numpy().T.reshape(n, 13, 3)
    _explained(H.state_fields(g_root, g_dof, g_cf), H.state_fields(o_root, o_dof, o_cf), flat, params, root, dof, tau,
               mu, "rough trimesh host", terrain=ter["oracle"])


@pytest.mark.parametrize("kind", ["hound", "anymal", "cartpole"])
def test_link_kinematics_match_oracle(kind):
    n = 40
    if kind == "hound":
        art, flat = H.hound()
        root, dof, _, mu = H.hound_states(n, seed=21)
        params = H.HOUND_PARAMS
    elif kind == "anymal":
        art, flat = H.anymal()
        root, dof, _, mu = H.anymal_states(n, seed=21)
        params = H.ANYMAL_PARAMS
    else:
        art, flat = H.cartpole()
        rng = np.random.RandomState(21)
        root = np.zeros((n, 13)); root[:, 2] = 2.0; root[:, 6] = 1.0
        dof = rng.uniform(-1.5, 1.5, (n, 2, 2))
        mu = np.ones((n, flat["ns"]))
        params = H.CARTPOLE_PARAMS
    gym, sim = H.make_host_sim(kind, n, params)
    H.load_state_into(sim, root, dof, mu)
    from isaacgymenv_amd.isaacgym import gymtorch
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    jac_t = gymtorch.wrap_tensor(gym.acquire_jacobian_tensor(sim, kind))
    mm_t = gymtorch.wrap_tensor(gym.acquire_mass_matrix_tensor(sim, kind))
    gym.refresh_rigid_body_state_tensor(sim)
    gym.refresh_jacobian_tensors(sim)
    gym.refresh_mass_matrix_tensors(sim)
    o_rb, o_jac, o_mm = KO.batch(flat, root, dof)
    g_rb = rb.numpy().astype(np.float64)
    nv = flat["nd"] + (0 if flat["fixed_base"] else 6)
    if flat["fixed_base"]:
        g_jac = np.concatenate([np.zeros((n, 1, 6, nv)), jac_t.numpy()], axis=1)
    else:
        g_jac = jac_t.numpy().astype(np.float64)
    np.testing.assert_allclose(g_rb[:, 0:3], o_rb[:, 0:3], atol=2e-5, rtol=1e-5)
    dots = np.abs(np.sum(g_rb[:, 3:7] * o_rb[:, 3:7], axis=1))
    assert dots.min() >= 1 - 1e-6, dots.min()
    np.testing.assert_allclose(g_rb[:, 7:13], o_rb[:, 7:13], atol=1e-4, rtol=1e-4)
    np.testing.assert_allclose(g_jac, o_jac, atol=2e-5, rtol=1e-5)
    np.testing.assert_allclose(mm_t.numpy(), o_mm, atol=1e-4, rtol=1e-4)


def test_thread_count_is_bit_invariant():
    n = 200
    art, flat = H.anymal()
    root, dof, tau, mu = H.anymal_states(n, seed=8, spread=2.0)
    outs = []
    for threads in (1, 3, 8):
        _, sim, g_root, g_dof = _host("anymal", n, H.ANYMAL_PARAMS, root, dof, tau, mu, 12, steps=5, threads=threads)
        outs.append((g_root, g_dof, sim.cf_soa.numpy().copy()))
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            np.testing.assert_array_equal(a, b)


def test_fused_step_equals_unfused_calls_on_host():
    """gs_sim_pd_step on the host backend == PD torque + simulate x4 + refresh dof, + 1 simulate."""
    n = 64
    art, flat = H.anymal()
    root, dof, _, mu = H.anymal_states(n, seed=4)
    q0 = np.array([H.ANYMAL_DEFAULT[d] for d in art.dof_names()], dtype=np.float32)
    actions = torch.from_numpy(np.random.RandomState(0).uniform(-1, 1, (n, 12)).astype(np.float32))
    res = {}
    for mode in ("fused", "unfused"):
        gym, sim = H.make_host_sim("anymal", n, H.ANYMAL_PARAMS)
        H.load_state_into(sim, root, dof, mu)
        gym.refresh_dof_state_tensor(sim)
        dpos = torch.from_numpy(q0)
        torques = torch.zeros(n, 12)
        if mode == "fused":
            gym.amd_pd_decimation_step(sim, actions, dpos, 80.0, 2.0, 0.5, 80.0, 4, 1, torques)
        else:
            dof_t = sim.dof_tensor.view(n, 12, 2)
            for _ in range(4):
                torques = torch.clip(80.0 * (0.5 * actions + dpos - dof_t[..., 0]) - 2.0 * dof_t[..., 1], -80., 80.)
                sim.dof_force.copy_(torques.reshape(-1))
                gym.simulate(sim)
                gym.refresh_dof_state_tensor(sim)
            gym.simulate(sim)
            gym.refresh_actor_root_state_tensor(sim)
            gym.refresh_net_contact_force_tensor(sim)
        res[mode] = (sim.state.numpy().copy(), sim.dof_tensor.numpy().copy(), sim.root_tensor.numpy().copy(),
                     sim.contact_tensor.numpy().copy(), torques.numpy().copy())
    for a, b in zip(res["fused"], res["unfused"]):
        np.testing.assert_allclose(a, b, atol=1e-5, rtol=1e-5)


def test_cartpole64_cpu_pipeline_tracks_oracle(monkeypatch):
    """BASELINE config 1 end to end: isaacgymenvs.make(task=Cartpole, num_envs=64, sim_device=cpu,
    pipeline=cpu), 600 env steps (past the 500-step timeout); each step's physics vs an oracle
    simulate from the state the sim held before the step."""
    from isaacgymenv_amd.isaacgymenvs.tasks.base import vec_task
    monkeypatch.setattr(vec_task, "EXISTING_SIM", None)
    import isaacgymenvs
    n = 64
    env = isaacgymenvs.make(seed=42, task="Cartpole", num_envs=n, sim_device="cpu", rl_device="cpu", headless=True,
                            overrides=["pipeline=cpu"])
    assert env.device == "cpu" and env.sim.host and env.sim.kernel_variant == 3
    assert env.sim.cparams.num_threads == 4  # physx.num_threads, cfg/config.yaml:30
    art, flat = H.cartpole()
    osim = OracleSim(flat, H.CARTPOLE_PARAMS)
    gen = torch.Generator().manual_seed(5)
    for t in range(600):
        before_root, before_dof = H.read_state(env.sim, 2)
        actions = 2 * torch.rand((n, 1), generator=gen) - 1
        obs, rew, reset, extras = env.step(actions)
        assert obs["obs"].shape == (n, 4) and obs["obs"].device.type == "cpu"
        assert reset.dtype == torch.int64 and extras["time_outs"].dtype == torch.bool
        assert int(env.progress_buf.max()) <= 499  # reset at progress >= max_episode_length - 1
        # the physics of this step, for the envs that were not reset inside post_physics_step
        tau = np.zeros((n, 2)); tau[:, 0] = actions.numpy()[:, 0] * 400.0
        r, d = before_root.copy(), before_dof.copy()
        osim.simulate(r, d, np.ascontiguousarray(tau), np.ones((n, flat["ns"])))
        _, g_dof = H.read_state(env.sim, 2)
        kept = (env.progress_buf.numpy() != 0)
        np.testing.assert_allclose(g_dof[kept], d[kept], atol=1e-4, rtol=1e-4, err_msg=f"step {t}")
        # observation = the refreshed dof tensor, clamped at clipObservations 5 (Cartpole.yaml:14)
        exp = np.stack([g_dof[:, 0, 0], g_dof[:, 0, 1], g_dof[:, 1, 0], g_dof[:, 1, 1]], axis=1)
        np.testing.assert_allclose(obs["obs"].numpy(), np.clip(exp, -5, 5), atol=1e-6)


def test_cartpole_reward_and_done_reproduce_golden_outputs():
    """Dynamics-free pin of the CPU pipeline's tail: compute_cartpole_reward on the fixture's own
    observations gives the reference's rewards and fall resets (tests/golden/cartpole.npz)."""
    from isaacgymenv_amd.isaacgymenvs.tasks.cartpole import compute_cartpole_reward
    d = np.load(os.path.join(GOLDEN, "cartpole.npz"))
    obs = torch.from_numpy(d["obs"]).double()
    checked = 0
    for t in range(obs.shape[0]):
        o = obs[t]
        inside = (o.abs() < 5.0).all(dim=1)  # the returned obs are clamped at 5; the reward used raw values
        rew, reset = compute_cartpole_reward(o[:, 2], o[:, 3], o[:, 1], o[:, 0], 3.0,
                                             torch.zeros(o.shape[0], dtype=torch.long),
                                             torch.zeros(o.shape[0], dtype=torch.long), 500.0)
        m = inside.numpy()
        np.testing.assert_allclose(rew.numpy()[m], d["rew"][t][m], rtol=1e-5, atol=1e-6, err_msg=f"step {t}")
        fell = d["reset"][t].astype(bool) & ~d["time_outs"][t].astype(bool)
        np.testing.assert_array_equal(reset.numpy()[m].astype(bool), fell[m], err_msg=f"step {t}")
        checked += int(m.sum())
    assert checked > 80  # envs whose returned observation is unclamped


def test_self_contact_pools_match_oracle_in_float():
    """The float narrowphase (gs_pairs.h, the source the GPU kernels run) against the fp64 oracle's pools on 512
    random UsefulHound states (arm anywhere in its limits: hull-hull, hull-cylinder, box-hull pairs): the same
    pairs in every env, and per contact the separation within 1e-5 m and the normal within a small angle.  Round 5
    (VERDICT r04 next 1): before the GJK fixes of DESIGN.md 3.12 the float search stalled on cylinder rims and on
    sliver simplices of two hulls -- 3 pool mismatches in 2048 states, separations off by up to 1.7 mm, 234 normals
    beyond 0.05 degrees."""
    n = 512
    art, flat = H.hound()
    root, dof, _, mu = H.hound_states(n, seed=5, spread=1.0)
    c64, k64 = OracleSim(flat, H.HOUND_PARAMS).self_contacts(root, dof, mu)
    gym, sim = H.make_host_sim("hound", n, H.HOUND_PARAMS, threads=8)
    H.load_state_into(sim, root, dof, mu)
    ch, kh = H.sim_self_contacts(sim, 0)
    ang, sep = [], []
    for e in range(n):
        a = [(int(c64[e, j, 8]), int(c64[e, j, 9])) for j in range(k64[e])]
        b = [(int(ch[e, j, 8]), int(ch[e, j, 9])) for j in range(kh[e])]
        assert a == b, (e, a, b)
        for j in range(kh[e]):
            ang.append(np.degrees(np.arccos(np.clip(np.dot(c64[e, j, 3:6], ch[e, j, 3:6]), -1.0, 1.0))))
            sep.append(abs(c64[e, j, 6] - ch[e, j, 6]))
    ang, sep = np.array(ang), np.array(sep)
    assert ang.size > 1000
    assert sep.max() <= 1e-5, sep.max()
    assert np.quantile(ang, 0.99) <= 0.1 and ang.max() <= 2.0, (np.quantile(ang, 0.99), ang.max())


def test_hound_fused_pd_step_random_states_match_oracle():
    """The r04f GPU failure's case on the host backend (same solver / narrowphase source): random UsefulHound states
    (seed 13, spread 0.5), actions RandomState(2), the fused 4 x PD + 1 sequence against the fp64 oracle, every
    env within the 5-substep tolerance or explained by the oracle's own perturbed spread."""
    n = 256
    art, flat = H.hound()
    root, dof, _, mu = H.hound_states(n, seed=13, spread=0.5)
    act = np.random.RandomState(2).uniform(-1.0, 1.0, (n, 18))
    default = np.array([0.0, 0.7854, -1.5708] * 4 + [0.0] * 6)
    kp, kd, scale = 80.0, 2.0, 0.5
    gym, sim = H.make_host_sim("hound", n, H.HOUND_PARAMS, threads=8)
    H.load_state_into(sim, root, dof, mu)
    gym.refresh_dof_state_tensor(sim)
    torques = torch.empty((n, 18))
    gym.amd_pd_decimation_step(sim, torch.from_numpy(act.astype(np.float32)),
                               torch.from_numpy(default.astype(np.float32)), kp, kd, scale, 80.0, 4, 1, torques)
    g_root, g_dof = H.read_state(sim, 18)
    got = dict(q=g_dof[:, :, 0], qd=g_dof[:, :, 1], pose=g_root[:, :7], vel=g_root[:, 7:],
               tau=torques.double().numpy(), cf=sim.contact_tensor.double().numpy().reshape(n, 24, 3))

    def seq(r0, d0, m, a, bits=64):
        dt = np.float64 if bits == 64 else np.float32
        osim = OracleSim(flat, H.HOUND_PARAMS, real_bits=bits)
        r, d = np.array(r0, dtype=dt), np.array(d0, dtype=dt)  # copies: the oracle steps them in place
        cf = np.zeros((r.shape[0], 24, 3), dt)
        tau = None
        for i in range(5):
            if i < 4:
                q, qd = d[:, :, 0].astype(np.float64), d[:, :, 1].astype(np.float64)
                tau = np.clip(kp * (scale * a + default - q) - kd * qd, -80.0, 80.0)
            osim.simulate(r, d, np.ascontiguousarray(tau, dtype=dt), np.ascontiguousarray(m, dtype=dt), cf)
        f = lambda x: np.asarray(x, np.float64)  # noqa: E731
        return dict(q=f(d[:, :, 0]), qd=f(d[:, :, 1]), pose=f(r[:, :7]), vel=f(r[:, 7:]), tau=f(tau), cf=f(cf))

    ref = seq(root, dof, mu, act)
    assert np.abs(ref["cf"]).sum() > 0

    def rerun(idx, rng, bits):
        r, d = H.perturbed(root, dof, idx, rng)
        return seq(r, d, mu[idx], act[idx], bits)
    tol = {"q": (1e-4, 0.0), "qd": (2.5e-2, 2.5e-2), "pose": (1e-4, 0.0), "vel": (2.5e-2, 2.5e-2),
           "tau": (0.5, 1e-2), "cf": (2.0, 5e-2)}
    H.assert_close_or_explained(got, ref, rerun, tol=tol, max_env_frac=0.03,
                                what="hound host fused 4 x PD + 1 (random states) vs oracle")


def test_fixed_base_planar_chain_on_ground_stays_finite():
    """a ground row the articulation cannot move along (J M^-1 J^T == 0) must take no impulse, not
    0 * inf.  Cartpole (fixed rail, cart sliding along y, pole hinged about x) lowered so that the cart's box
    corners sit 5 mm inside the plane: the cart can move neither along x nor along z, so those rows have zero
    response.  Host backend and oracle stay finite, agree, and put no force on the cart."""
    n = 8
    art, flat = H.cartpole()
    params = dict(H.CARTPOLE_PARAMS, collect_contacts=1)
    root = np.zeros((n, 13)); root[:, 2] = 0.095; root[:, 6] = 1.0
    dof = np.zeros((n, 2, 2))
    dof[:, 0, 1] = np.linspace(-1.0, 1.0, n)
    dof[:, 1, 0] = np.linspace(-0.3, 0.3, n)
    tau = np.zeros((n, 2)); mu = np.ones((n, flat["ns"]))
    gym, sim, g_root, g_dof = _host("cartpole", n, params, root, dof, tau, mu, 2, steps=3)
    o_root, o_dof, o_cf = _oracle(flat, params, root, dof, tau, mu, steps=3)
    assert np.isfinite(o_dof).all() and np.isfinite(g_dof).all()
    np.testing.assert_allclose(g_dof, o_dof, atol=1e-4, rtol=1e-4)
    gym.refresh_net_contact_force_tensor(sim)
    g_cf = sim.contact_tensor.numpy().reshape(n, flat["nr"], 3)
    assert np.isfinite(g_cf).all()
    np.testing.assert_array_equal(g_cf[:, 1], 0.0)  # the cart (body 1): every row has zero response
    np.testing.assert_array_equal(o_cf[:, 1], 0.0)


def test_terrain_query_on_jittered_mesh_matches_oracle():
    """the cell cull of gs_terrain.h must bound every vertex the mesh check admits, not only the
    terrain_utils moves of exactly one cell.  A heightfield-grid mesh whose vertices are jittered off their grid
    points by up to 0.2 cells in x and y (and a few by a whole cell), queried at 100k random spheres on the host
    backend (the same gs_terrain.h source as the kernels) against the oracle's scan of every cell in range, which
    culls nothing."""
    from isaacgymenv_amd.isaacgym import _lib, terrain_utils
    rng = np.random.RandomState(9)
    rows, cols, hs = 60, 60, 0.1
    hf = (rng.randint(-12, 12, (rows, cols)) * 4).astype(np.int16)
    v, t = terrain_utils.convert_heightfield_to_trimesh(hf, hs, 0.005, None)
    v = v.astype(np.float64)
    v[:, :2] += rng.uniform(-0.2, 0.2, (v.shape[0], 2)) * hs
    whole = rng.rand(v.shape[0]) < 0.02
    v[whole, 0] += np.where(rng.rand(whole.sum()) < 0.5, -1.0, 1.0) * hs * 0.75
    grid = v.reshape(rows, cols, 3)
    # the outer rows' x and columns' y on their grid lines: they define the grid origin and spacing
    grid[0, :, 0], grid[-1, :, 0] = 0.0, (rows - 1) * hs
    grid[:, 0, 1], grid[:, -1, 1] = 0.0, (cols - 1) * hs
    ter = H.mesh_terrain(v.astype(np.float32), t, rows, cols, hs, shift=(-3.0, -3.0, 0.0))
    art, flat = H.anymal()
    params = dict(H.ANYMAL_PARAMS, has_ground=0)
    gym, sim = H.make_host_sim("anymal", 1, params, terrain=ter)
    o = ter["oracle"]
    n = 100000
    c = np.zeros((n, 3))
    c[:, 0] = rng.uniform(o["x0"] + 0.2, o["x0"] + (rows - 2) * hs - 0.2, n)
    c[:, 1] = rng.uniform(o["y0"] + 0.2, o["y0"] + (cols - 2) * hs - 0.2, n)
    gi = np.clip(np.round((c[:, 0] - o["x0"]) / hs).astype(int), 0, rows - 1)
    gj = np.clip(np.round((c[:, 1] - o["y0"]) / hs).astype(int), 0, cols - 1)
    c[:, 2] = o["vertices"].reshape(rows, cols, 3)[gi, gj, 2] + rng.uniform(-0.1, 0.15, n)
    r = rng.choice([0.02, 0.05, 0.1], n)
    cf, rf = c.astype(np.float32), r.astype(np.float32)
    out = np.zeros((n, 5), np.float32)
    _lib.check(_lib.lib().gs_debug_terrain_query(sim.handle, cf.ctypes.data, rf.ctypes.data, n, out.ctypes.data,
                                                 None), "terrain query")
    ref = OracleSim(flat, params, terrain=o).terrain_query(cf.astype(np.float64), rf.astype(np.float64))
    found_g, found_o = out[:, 0] > 0.5, ref[:, 0] > 0.5
    assert found_o.mean() > 0.3
    assert (found_g != found_o).mean() < 2e-4
    both = found_g & found_o
    dsep = np.abs(out[both, 1] - ref[both, 1])
    assert (dsep > 1e-4).mean() < 5e-4, ((dsep > 1e-4).mean(), dsep.max())


def test_cylinder_end_near_ground_is_not_skipped():
    """Round 5, found by the 4096-env UsefulHound parity test (tests/test_baseline_sizes_gpu.py, env 680 of a state
    the task reached after 30 steps, fixture tests/golden/hound_cylinder_ground_case.npz): the solver skips a shape
    whose bounding sphere clears the ground, but a cylinder's ground candidates are capsule ends (hl + r from the
    centre) that reach beyond the cylinder's own bounding sphere sqrt(hl^2 + r^2).  A leg cylinder's end 10 mm from
    the ground was skipped at a 42 mm sphere clearance; the spinning robot's contact impulse was lost (q off by
    8e-4 rad in one simulate).  gs_sim_set_model now widens each shape's sphere to its candidates."""
    z = np.load(os.path.join(GOLDEN, "hound_cylinder_ground_case.npz"))
    root, dof, mu, tau = z["root"], z["dof"], z["mu"], z["tau"]
    art, flat = H.hound()
    for params in (H.HOUND_PARAMS, dict(H.HOUND_PARAMS, pos_iters=1, vel_iters=0)):
        _, sim, g_root, g_dof = _host("hound", 1, params, root, dof, tau, mu, 18)
        o_root, o_dof, _, _ = H.oracle_run(flat, params, root, dof, tau, mu, nc=24)
        np.testing.assert_allclose(g_dof[:, :, 0], o_dof[:, :, 0], atol=2e-6)
        np.testing.assert_allclose(g_dof[:, :, 1], o_dof[:, :, 1], atol=5e-4, rtol=1e-4)
        np.testing.assert_allclose(g_root[:, 7:], o_root[:, 7:], atol=5e-4, rtol=1e-4)


def test_host_tgs_matches_oracle_tgs_and_warns_nothing():
    """physx.solver_type 1 on the host backend (the lane solver source, gs_solver.h): one simulate from random ANYmal
    states and from Ant states (joint limits + force sensors) against the oracle's TGS (solver_type 3), the GPU
    tolerances through the explained-env rule; no PhysicsDeviationWarning (TGS is simulated)."""
    import warnings
    from isaacgymenv_amd.isaacgym.gymapi import PhysicsDeviationWarning
    for kind, mk, states, params, nd in (("anymal", H.anymal, H.anymal_states, H.ANYMAL_PARAMS, 12),
                                         ("ant", H.ant, H.ant_states, H.ANT_PARAMS, 8)):
        n = 64
        art, flat = mk()
        root, dof, tau, mu = states(n, seed=6)
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            gym, sim = H.make_host_sim(kind, n, dict(params, solver_type=1), threads=2)
        assert not any(issubclass(x.category, PhysicsDeviationWarning) for x in w), kind
        assert sim.cparams.solver_type == 1
        H.load_state_into(sim, root, dof, mu)
        sim.dof_force.copy_(torch.from_numpy(tau.astype(np.float32).reshape(-1)))
        gym.simulate(sim)
        g_root, g_dof = H.read_state(sim, nd)
        op = dict(params, solver_type=3)
        o_root, o_dof, _, _ = H.oracle_run(flat, op, root, dof, tau, mu)

        def rerun(idx, rng, bits=64):
            r, d = H.perturbed(root, dof, idx, rng)
            rr, dd, _, _ = H.oracle_run(flat, op, r, d, tau[idx], mu[idx], bits=bits)
            return H.state_fields(rr, dd)

        H.assert_close_or_explained(H.state_fields(g_root, g_dof), H.state_fields(o_root, o_dof), rerun,
                                    what=f"host TGS one simulate vs the oracle's TGS ({kind}, {n} random states)")


def test_set_root_and_dof_in_one_call_equals_the_two_indexed_sets():
    """gs_sim_set_root_and_dof (ABI 9: a reset's root and dof indexed sets in one call / one launch) writes the same
    sim state as gs_sim_set_root then gs_sim_set_dof with the same indices (host backend; the GPU form runs in every
    fused reset of tests/test_task_gpu.py)."""
    import torch
    art, flat = H.anymal()
    n = 16
    rng = np.random.RandomState(4)
    sims = [H.make_host_sim("anymal", n, H.ANYMAL_PARAMS)[1] for _ in range(2)]
    root = torch.from_numpy(rng.normal(size=(n, 13)).astype(np.float32))
    root[:, 3:7] /= root[:, 3:7].norm(dim=1, keepdim=True)
    dof = torch.from_numpy(rng.normal(size=(n * 12, 2)).astype(np.float32))
    idx = torch.tensor([1, 4, 5, 11, 15], dtype=torch.int32)
    sims[0].set_root_and_dof(root, dof, idx, len(idx))
    sims[1].set_state("root", root, idx, len(idx))
    sims[1].set_state("dof", dof, idx, len(idx))
    assert torch.equal(sims[0].state, sims[1].state)
    untouched = [e for e in range(n) if e not in idx.tolist()]
    fresh = H.make_host_sim("anymal", n, H.ANYMAL_PARAMS)[1].state
    assert torch.equal(sims[0].state[:, untouched], fresh[:, untouched])
