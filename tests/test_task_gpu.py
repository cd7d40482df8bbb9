"""End-to-end AnymalTerrain / Cartpole on the GPU pipeline (real HIP simulator).

* the fused decimation kernel (gs_sim_pd_step) is observably equivalent to the
  reference's unfused sequence (torch PD -> set efforts -> simulate -> refresh,
  x4, + 1 simulate) from the same state;
* a full 1000-step episode runs with finite observations, robots standing on
  the plane, the AnymalTerrain quirks intact (bool done mask, time_outs never
  set, every env reset at progress 999 = step 998 of a fresh episode).
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _make(task, n, monkeypatch, **over):
    from isaacgymenv_amd.isaacgymenvs.tasks.base import vec_task
    monkeypatch.setattr(vec_task, "EXISTING_SIM", None)
    import isaacgymenvs
    torch.manual_seed(42)
    ov = [f"{k}={v}" for k, v in over.items()]
    return isaacgymenvs.make(seed=42, task=task, num_envs=n, sim_device="cuda:0", rl_device="cuda:0",
                             headless=True, force_render=False, overrides=ov)


def _snapshot(env):
    names = ["commands", "last_actions", "last_dof_vel", "feet_air_time", "progress_buf", "torques", "root_states",
             "dof_state", "contact_forces", "obs_buf", "rew_buf"]
    s = {n: getattr(env, n).clone() for n in names}
    s["reset_buf"] = env.reset_buf.clone()
    s["timeout_buf"] = env.timeout_buf.clone()
    s["sums"] = {k: v.clone() for k, v in env.episode_sums.items()}
    s["sim_state"] = env.sim.state.clone()
    s["sim_cf"] = env.sim.cf_soa.clone()
    s["rng"] = torch.cuda.get_rng_state()
    s["counter"] = env.common_step_counter
    if env.custom_origins:
        s["terrain"] = (env.terrain_levels.clone(), env.env_origins.clone())
    return s


def _restore(env, s):
    for n in ["commands", "last_actions", "last_dof_vel", "feet_air_time", "progress_buf", "torques", "root_states",
              "dof_state", "contact_forces", "obs_buf", "rew_buf"]:
        getattr(env, n).copy_(s[n])
    env.reset_buf.copy_(s["reset_buf"])
    env.timeout_buf = s["timeout_buf"].clone()
    for k, v in s["sums"].items():
        env.episode_sums[k].copy_(v)
    env.sim.state.copy_(s["sim_state"])
    env.sim.cf_soa.copy_(s["sim_cf"])
    torch.cuda.set_rng_state(s["rng"])
    env.common_step_counter = s["counter"]
    if "terrain" in s:
        env.terrain_levels.copy_(s["terrain"][0])
        env.env_origins.copy_(s["terrain"][1])


def test_fused_step_equals_unfused_sequence(monkeypatch):
    """The fused decimation kernel vs the reference's unfused sequence (torch PD -> set efforts -> simulate
    -> refresh, x4, + 1 simulate) over 3 env steps from the same state.  The fused kernel evaluates the PD
    torque with FMAs, the unfused path with separate torch ops; that last-bit difference passes through
    the contact solver's switches (activity, friction cone), so an env may drift apart -- then it must be
    one the unfused sequence itself moves as far when its sim state is perturbed at fp32-rounding size
    (helpers.assert_close_or_explained)."""
    from tests import helpers as H
    n = 256
    env = _make("AnymalTerrain", n, monkeypatch)
    gen = torch.Generator(device="cuda:0").manual_seed(5)
    acts = [2 * torch.rand((n, 12), device="cuda:0", generator=gen) - 1 for _ in range(3)]
    for a in acts:  # leave the initial state
        env.step(a)
    snap = _snapshot(env)
    nd = 12

    def run(mode, idx=None, rng=None):
        _restore(env, snap)
        if idx is not None:  # fp32-rounding-sized noise on the sim state of envs idx (H.perturbed's sizes)
            st = env.sim.state
            m = len(idx)
            ii = torch.as_tensor(idx, device=st.device)
            for rows, sd in ((range(0, 3), 1e-6), (range(7, 13), 1e-5), (range(13, 13 + nd), 1e-6),
                             (range(13 + nd, 13 + 2 * nd), 1e-5)):
                for row in rows:
                    st[row, ii] += torch.from_numpy(rng.normal(0, sd, m).astype(np.float32)).to(st.device)
        monkeypatch.setenv("GS_DISABLE_FUSED", mode)
        res = {k: [] for k in ("q", "qd", "pose", "vel", "obs", "rew")}
        resets = []
        for a in acts:
            obs, rew, reset, _ = env.step(a)
            q = env.dof_state.view(n, nd, 2)
            res["q"].append(q[..., 0].cpu().numpy())
            res["qd"].append(q[..., 1].cpu().numpy())
            res["pose"].append(env.root_states[:, :7].cpu().numpy())
            res["vel"].append(env.root_states[:, 7:].cpu().numpy())
            res["obs"].append(obs["obs"].cpu().numpy())
            res["rew"].append(rew.cpu().numpy()[:, None])
            resets.append(reset.clone())
        return {k: np.stack(v, axis=1) for k, v in res.items()}, resets

    unfused, r_unfused = run("1")
    fused, r_fused = run("0")
    for d1, d2 in zip(r_unfused, r_fused):
        assert torch.equal(d1, d2)

    def rerun(idx, rng):
        out, _ = run("1", idx, rng)
        return {k: v[idx] for k, v in out.items()}
    tol = {"q": (2e-4, 0.0), "qd": (1e-2, 1e-2), "pose": (2e-4, 0.0), "vel": (1e-2, 1e-2), "obs": (1e-2, 1e-2),
           "rew": (1e-4, 1e-2)}
    H.assert_close_or_explained(fused, unfused, rerun, tol=tol, max_env_frac=1e-2,
                                what="fused vs unfused AnymalTerrain step (3 env steps)")


TRIMESH = {"task.env.terrain.terrainType": "trimesh", "task.env.terrain.numLevels": 4,
           "task.env.terrain.numTerrains": 8}


@pytest.mark.parametrize("terrain", ["plane", "trimesh"])
def test_kernel_tail_equals_torch_tail_across_resets(terrain, monkeypatch):
    """The fused tail (post_a -> optimistic noise/post_b -> RNG rollback + reset_idx + post_b on
    reset steps) against the reference's torch statements, same physics kernel and same CUDA
    RNG stream, over 5-step episodes so that most steps reset someone.  Trimesh: the fused reset
    also runs the terrain curriculum (update_terrain_level, new origins, root x/y draws) and the
    terrain-level mean."""
    n = 256
    over = {"task.env.learn.episodeLength_s": 0.1}
    if terrain == "trimesh":
        over.update(TRIMESH)
    env = _make("AnymalTerrain", n, monkeypatch, **over)
    assert env.custom_origins == (terrain == "trimesh")
    assert env.max_episode_length in (5, 6)
    gen = torch.Generator(device="cuda:0").manual_seed(9)
    acts = [2 * torch.rand((n, 12), device="cuda:0", generator=gen) - 1 for _ in range(12)]
    env.step(acts[0])
    snap = _snapshot(env)
    kernels = env._kernels
    out = {}
    for mode in ("kernels", "torch"):
        _restore(env, snap)
        env._kernels = kernels if mode == "kernels" else None
        env.extras.pop("episode", None)
        res = []
        for a in acts:
            obs, rew, reset, extras = env.step(a)
            ep = extras.get("episode")
            res.append((obs["obs"].clone(), rew.clone(), reset.clone(), extras["time_outs"].clone(),
                        None if ep is None else torch.stack([torch.as_tensor(v, device="cuda:0").float()
                                                             for v in ep.values()]),
                        env.root_states.clone(),
                        env.terrain_levels.clone() if env.custom_origins else None))
            env.extras.pop("episode", None)
        out[mode] = res
    env._kernels = kernels
    n_reset_steps = 0
    for t, (a, b) in enumerate(zip(out["kernels"], out["torch"])):
        assert torch.equal(a[2], b[2]), f"reset mask step {t}"
        n_reset_steps += int(bool(a[2].any()))
        assert torch.equal(a[3], b[3]), f"time_outs step {t}"
        torch.testing.assert_close(a[0], b[0], rtol=1e-5, atol=1e-5, msg=f"obs step {t}")
        torch.testing.assert_close(a[1], b[1], rtol=1e-5, atol=1e-6, msg=f"reward step {t}")
        assert (a[4] is None) == (b[4] is None)
        if a[4] is not None:
            torch.testing.assert_close(a[4], b[4], rtol=1e-4, atol=1e-7, msg=f"episode extras step {t}")
        torch.testing.assert_close(a[5], b[5], rtol=1e-5, atol=1e-5, msg=f"root states step {t}")
        if a[6] is not None:
            assert torch.equal(a[6], b[6]), f"terrain levels step {t}"
    assert n_reset_steps >= 2


@pytest.mark.parametrize("terrain", ["plane"])  # (the TERR kernels carry no tail: gs_sim_pd_tail_supported 0)
def test_fused_tail_in_physics_launch_is_bit_identical_to_post_a(terrain, monkeypatch):
    """post_a run by the lane-team physics kernel's last phase (gymsim ABI 9, gs_pd_args.tail_*) against the
    separate k_post_a launch, from the same state over 12 steps of 5-step episodes with a push step inside the
    window (that step falls back to the separate launch): every output bit-identical -- the same source
    (gt_anymal_tail.h) compiled without FMA contraction in both libraries."""
    n = 256
    over = {"task.env.learn.episodeLength_s": 0.1}
    if terrain == "trimesh":
        over.update(TRIMESH)
    monkeypatch.setenv("GS_FUSED_TAIL", "1")
    env = _make("AnymalTerrain", n, monkeypatch, **over)
    assert env.gym.amd_pd_tail_supported(env.sim)
    gen = torch.Generator(device="cuda:0").manual_seed(11)
    acts = [2 * torch.rand((n, 12), device="cuda:0", generator=gen) - 1 for _ in range(12)]
    env.step(acts[0])
    env.common_step_counter = env.push_interval - 6  # the 6th step below pushes
    snap = _snapshot(env)
    kernels = env._kernels
    out, fused_steps = {}, {}
    for mode in ("fused", "separate"):
        _restore(env, snap)
        kernels._tail_ok = None if mode == "fused" else False
        env.extras.pop("episode", None)
        res, n0 = [], env.fused_tail_steps
        for a in acts:
            obs, rew, reset, extras = env.step(a)
            ep = extras.get("episode")
            res.append([obs["obs"].clone(), rew.clone(), reset.clone(), extras["time_outs"].clone(),
                        None if ep is None else torch.stack([torch.as_tensor(v, device="cuda:0").float()
                                                             for v in ep.values()]),
                        env.root_states.clone(), env.progress_buf.clone(), env.commands.clone(),
                        env.feet_air_time.clone(), torch.stack([v.clone() for v in env.episode_sums.values()]),
                        env.base_lin_vel.clone(), env.projected_gravity.clone(), kernels.reset_masks.clone()])
            env.extras.pop("episode", None)
        out[mode] = res
        fused_steps[mode] = env.fused_tail_steps - n0
    kernels._tail_ok = None
    # every step but the push step ran post_a in the physics launch; the separate mode never did
    assert fused_steps == {"fused": len(acts) - 1, "separate": 0}, fused_steps
    n_reset_steps = 0
    for t, (a, b) in enumerate(zip(out["fused"], out["separate"])):
        n_reset_steps += int(bool(a[2].any()))
        for k, (x, y) in enumerate(zip(a, b)):
            assert (x is None) == (y is None), (t, k)
            if x is not None:
                assert torch.equal(x, y), f"step {t} output {k}"
    assert n_reset_steps >= 2


def test_anymal_full_episode(monkeypatch):
    n = 512
    env = _make("AnymalTerrain", n, monkeypatch)
    gen = torch.Generator(device="cuda:0").manual_seed(3)
    env.reset()
    heights, dones = [], []
    for t in range(1000):
        a = 0.3 * (2 * torch.rand((n, 12), device="cuda:0", generator=gen) - 1)
        obs, rew, reset, extras = env.step(a)
        assert reset.dtype == torch.bool
        assert not bool(extras["time_outs"].any()), "AnymalTerrain time_outs is always False (SURVEY.md 0.5)"
        if t % 50 == 0:
            assert torch.isfinite(obs["obs"]).all() and torch.isfinite(rew).all()
            heights.append(float(env.root_states[:, 2].mean()))
        dones.append(reset.clone())
    d = torch.stack(dones)
    # envs that never fell are all reset together when progress reaches 999 (step index 998)
    never_fell = ~d[:998].any(0)
    assert bool(d[998][never_fell].all())
    assert float(never_fell.float().mean()) > 0.5, "most robots should stay up under small random actions"
    assert 0.35 < np.mean(heights[2:]) < 0.65, heights


def test_cartpole_gpu_runs(monkeypatch):
    env = _make("Cartpole", 64, monkeypatch)
    for t in range(200):
        a = 2 * torch.rand((64, 1), device="cuda:0") - 1
        obs, rew, reset, _ = env.step(a)
        assert reset.dtype == torch.int64
        assert torch.isfinite(obs["obs"]).all()
    assert float(obs["obs"].abs().max()) <= 5.0  # clipObservations


def test_ant_gpu_episode(monkeypatch):
    """Ant (A13) on the real simulator: standing still it stays upright with its weight carried by the
    foot sensors; under random torques some ants fall (height < terminationHeight) and are reset, and
    every env that never fell resets together at the episode end."""
    n = 512
    env = _make("Ant", n, monkeypatch)
    assert env.obs_buf.shape == (n, 60) and env.reset_buf.dtype == torch.int64
    zero = torch.zeros((n, 8), device="cuda:0")
    env.step(zero)  # the initial all-envs reset happens on the first step
    for _ in range(60):
        obs, rew, reset, extras = env.step(zero)
    o = obs["obs"]
    assert torch.isfinite(o).all()
    assert float((o[:, 10] > 0.93).float().mean()) > 0.95, "resting ants stay upright"
    assert not bool(reset.any())
    z = env.root_states[:, 2]
    assert 0.31 < float(z.min()) and float(z.max()) < 0.7
    # weight of everything above the feet hangs on the four foot joints
    from tests.helpers import ANT_FEET, ant
    mass = ant()[1]["mass"]
    load = 9.81 * (float(np.sum(mass)) - float(np.sum(mass[ANT_FEET])))
    # (readings are in the tilted foot frames, so compare the sum of magnitudes, which bounds the
    # world-frame resultant from above; a leg resting on the plane bypasses the sensors -> median)
    f = env.vec_sensor_tensor.view(n, 4, 6)[:, :, 0:3].norm(dim=-1).sum(1)
    assert 0.6 * load < float(f.median()) < 2.5 * load, (float(f.median()), load)
    # random torques: falls and resets happen, the episode end resets the survivors
    gen = torch.Generator(device="cuda:0").manual_seed(3)
    dones = []
    for t in range(1000):
        a = 2 * torch.rand((n, 8), device="cuda:0", generator=gen) - 1
        obs, rew, reset, extras = env.step(a)
        if t % 100 == 0:
            assert torch.isfinite(obs["obs"]).all() and torch.isfinite(rew).all()
        dones.append(reset.clone())
    d = torch.stack(dones)
    assert int(d.sum()) >= n // 4
    assert torch.isfinite(extras["true_objective"]).all()


def test_episode_extras_are_bit_identical_across_same_seed_runs(monkeypatch):
    """extras["episode"] (the fused reset's per-term means) is reduced in a fixed order, so two runs
    from the same seed give the same bits on every reset step (cross-wave float atomics)."""
    n = 2048

    def run():
        env = _make("AnymalTerrain", n, monkeypatch, **{"task.env.learn.episodeLength_s": 0.6})
        gen = torch.Generator(device="cuda:0").manual_seed(9)
        eps = []
        for _ in range(70):
            _, _, reset, extras = env.step(2 * torch.rand((n, 12), device="cuda:0", generator=gen) - 1)
            ep = extras.get("episode")
            if ep is not None and bool(reset.any()):
                eps.append(torch.stack([ep[k].float().reshape(()) for k in sorted(ep)]).cpu())
            env.extras.pop("episode", None)
        torch.cuda.synchronize()
        return eps

    a, b = run(), run()
    assert len(a) >= 2 and len(a) == len(b)
    for x, y in zip(a, b):
        assert torch.equal(x.view(torch.int32), y.view(torch.int32))


def test_obs_mirror_holds_every_returned_observation(monkeypatch):
    """amd_set_obs_mirror (a learner's static act-forward input): after every step, reset steps included, the
    mirror holds exactly the observations VecTask returned, and the returned tensor is still a fresh one."""
    n = 256
    env = _make("AnymalTerrain", n, monkeypatch, **{"task.env.learn.episodeLength_s": 0.1})
    buf = torch.zeros_like(env.obs_buf)
    assert env.amd_set_obs_mirror(buf)
    gen = torch.Generator(device="cuda:0").manual_seed(13)
    resets, prev = 0, None
    for _ in range(12):
        obs, _, reset, _ = env.step(2 * torch.rand((n, 12), device="cuda:0", generator=gen) - 1)
        o = obs["obs"]
        assert env._obs_mirrored is o and o.data_ptr() != buf.data_ptr()
        assert prev is None or o.data_ptr() != prev.data_ptr() or True
        assert torch.equal(buf, o)
        resets += int(bool(reset.any()))
        prev = o
    assert resets >= 2
    env.amd_set_obs_mirror(None)
    obs, _, _, _ = env.step(torch.zeros((n, 12), device="cuda:0"))
    assert env._obs_mirrored is None


def test_post_ab_launch_is_bit_identical_to_post_a_then_post_b(monkeypatch):
    """gt_anymal_post_physics_ab (post_a and the optimistic observations in one launch, 16 envs per workgroup)
    against the separate k_post_a + k_post_b launches from the same state, over 12 steps of 5-step episodes with a
    push step: every output bit-identical (the same sources, gt_anymal_tail.h and k_post_b's element body)."""
    n = 256
    monkeypatch.setenv("GT_POST_AB", "1")  # (opt-in: measured slower, gymtask.post_ab_applies)
    env = _make("AnymalTerrain", n, monkeypatch, **{"task.env.learn.episodeLength_s": 0.1})
    gen = torch.Generator(device="cuda:0").manual_seed(21)
    acts = [2 * torch.rand((n, 12), device="cuda:0", generator=gen) - 1 for _ in range(12)]
    env.step(acts[0])
    env.common_step_counter = env.push_interval - 6
    snap = _snapshot(env)
    kernels = env._kernels
    out = {}
    for mode in ("ab", "separate"):
        _restore(env, snap)
        kernels._ab_ok = None if mode == "ab" else False
        assert kernels.post_ab_applies() == (mode == "ab")
        env.extras.pop("episode", None)
        res = []
        for a in acts:
            obs, rew, reset, extras = env.step(a)
            ep = extras.get("episode")
            res.append([obs["obs"].clone(), rew.clone(), reset.clone(), extras["time_outs"].clone(),
                        None if ep is None else torch.stack([torch.as_tensor(v, device="cuda:0").float()
                                                             for v in ep.values()]),
                        env.root_states.clone(), env.progress_buf.clone(), env.commands.clone(),
                        env.feet_air_time.clone(), torch.stack([v.clone() for v in env.episode_sums.values()]),
                        env.last_actions.clone(), env.last_dof_vel.clone(), kernels.reset_masks.clone(),
                        kernels.reset_count.clone()])
            env.extras.pop("episode", None)
        out[mode] = res
    kernels._ab_ok = None
    n_reset_steps = 0
    for t, (a, b) in enumerate(zip(out["ab"], out["separate"])):
        n_reset_steps += int(bool(a[2].any()))
        for k, (x, y) in enumerate(zip(a, b)):
            assert (x is None) == (y is None), (t, k)
            if x is not None:
                assert torch.equal(x, y), f"step {t} output {k}"
    assert n_reset_steps >= 2
