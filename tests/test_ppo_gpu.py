"""PPO learner on the GPU: the GAE HIP kernel (libgymrl.so) against the oracle (bit-exact),
and end-to-end training through the product path (Cartpole learning, AnymalTerrain epochs)."""
import numpy as np
import pytest
import torch

from oracle import ppo_oracle as O

pytestmark = pytest.mark.gpu


def _rollout(H, N, seed, done_p=0.05):
    rng = np.random.RandomState(seed)
    r = rng.randn(H, N).astype(np.float32)
    v = (rng.randn(H, N) * 10).astype(np.float32)
    d = (rng.rand(H, N) < done_p).astype(np.uint8)
    lv = rng.randn(N).astype(np.float32)
    ld = (rng.rand(N) < done_p).astype(np.uint8)
    return r, v, d, lv, ld


@pytest.mark.parametrize("H,N", [(24, 4096), (24, 4133), (1, 1), (16, 512), (240, 100), (7, 65)])
def test_gae_kernel_bit_exact(H, N):
    from isaacgymenv_amd.rl.gae import discount_values
    r, v, d, lv, ld = _rollout(H, N, seed=H + 7 * N)
    dev = [torch.from_numpy(x).cuda() for x in (r, v, d, lv, ld)]
    ret, adv, vals = discount_values(*dev, 0.99, 0.95)
    oadv = O.discount_values(r, v, d, lv, ld, 0.99, 0.95)
    np.testing.assert_array_equal(adv.cpu().numpy(), O.env_major(oadv))
    np.testing.assert_array_equal(ret.cpu().numpy(), O.env_major(oadv + v))
    np.testing.assert_array_equal(vals.cpu().numpy(), O.env_major(v))


def test_gae_kernel_rejects_oversized_horizon():
    from isaacgymenv_amd.rl.gae import discount_values
    H, N = 241, 8
    z = torch.zeros(H, N, device="cuda")
    with pytest.raises(RuntimeError, match="horizon"):
        discount_values(z, z, torch.zeros(H, N, dtype=torch.uint8, device="cuda"), torch.zeros(N, device="cuda"),
                        torch.zeros(N, dtype=torch.uint8, device="cuda"), 0.99, 0.95)


def _agent(task, num_envs, overrides=(), **over):
    from isaacgymenv_amd.isaacgymenvs.config import compose
    from isaacgymenv_amd.isaacgymenvs.tasks.base import vec_task
    from isaacgymenv_amd.rl import A2CAgent, PpoConfig
    import isaacgymenvs
    vec_task.EXISTING_SIM = None
    cfg = compose("config", [f"task={task}"])
    env = isaacgymenvs.make(seed=42, task=task, num_envs=num_envs, sim_device="cuda:0", rl_device="cuda:0",
                            headless=True, force_render=False, overrides=list(overrides))
    pcfg = PpoConfig.from_train_cfg(cfg["train"], **over)
    return A2CAgent(env, pcfg, device="cuda:0", seed=42)


def test_cartpole_ppo_learns():
    # (through the fused loss kernel, f32: CartpolePPO.yaml has no mixed precision, shared trunk)
    # rl_games solves Cartpole (episode 500 steps) in ~100 epochs; this learner reaches ~490 mean
    # episode length by epoch 60 (tools/probes/ppo_probe.py); random play lasts ~3 steps
    agent = _agent("Cartpole", 512)
    for ep in range(60):
        agent.train_epoch()
    s = agent.epoch_stats()
    assert s["mean_length"] > 250, s
    assert np.isfinite(s["kl"])


def test_anymal_terrain_ppo_epochs():
    agent = _agent("AnymalTerrain", 4096)
    assert agent.num_params * 4 == 2094692 and agent.num_minibatches == 6
    for _ in range(2):
        agent.train_epoch()
    s = agent.epoch_stats()
    assert np.isfinite(s["kl"]) and np.isfinite(s["a_loss"]) and np.isfinite(s["c_loss"])
    assert all(torch.isfinite(p).all() for p in agent.params)
    assert agent.frame == 2 * 24 * 4096


def test_anymal_terrain_trimesh_ppo_epochs():
    """BASELINE config 3: PPO on the trimesh heightfield (curriculum resets, mesh contacts, height probes)."""
    agent = _agent("AnymalTerrain", 4096, overrides=["task.env.terrain.terrainType=trimesh"])
    assert agent.env.cfg["env"]["terrain"]["terrainType"] == "trimesh" and agent.env.custom_origins
    for _ in range(3):  # the third epoch replays the captured graphs
        agent.train_epoch()
    s = agent.epoch_stats()
    assert np.isfinite(s["kl"]) and np.isfinite(s["a_loss"]) and np.isfinite(s["c_loss"])
    assert all(torch.isfinite(p).all() for p in agent.params)
    assert torch.isfinite(agent.env.obs_buf).all()
    assert agent.frame == 3 * 24 * 4096


def test_graph_replay_equals_eager_updates():
    """The HIP-graph path (captured after epoch 1) performs the same updates as the eager path."""
    runs = []
    for graphs in (False, True):
        torch.manual_seed(0)
        agent = _agent("Cartpole", 512)
        agent.use_graphs = graphs
        for _ in range(3):
            agent.train_epoch()
        assert (agent._mb_graphs is not None) == graphs
        runs.append((torch.cat([p.detach().reshape(-1) for p in agent.params]).cpu(), agent.epoch_stats(),
                     agent.b_obs.cpu()))
    (pe, se, oe), (pg, sg, og) = runs
    torch.testing.assert_close(og, oe, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(pg, pe, rtol=1e-3, atol=1e-5)
    assert abs(sg["lr"] - se["lr"]) <= 1e-9 + 1e-6 * se["lr"]


def test_act_graph_replay_equals_eager_forward():
    """The captured act forward (sampling noise drawn outside the graph into its static input) returns, from the
    same generator state, exactly the eager forward's outputs, and leaves the generator where the eager one does."""
    agent = _agent("AnymalTerrain", 1024, minibatch_size=8192)
    agent.train_epoch()  # eager epoch, then the graphs are captured
    assert agent._act_graph is not None and agent._g_noise is not None
    obs = agent.obs["obs"].clone()
    torch.manual_seed(5)
    got = {k: v.clone() for k, v in agent.get_action_values(obs).items()}
    off_graph = torch.cuda.default_generators[0].get_offset()
    torch.manual_seed(5)
    agent.model.eval()
    with torch.no_grad():
        ref = agent.model({"is_train": False, "obs": obs})
    assert torch.cuda.default_generators[0].get_offset() == off_graph
    for k in ("actions", "mus", "sigmas", "values", "neglogpacs"):
        assert torch.equal(got[k], ref[k]), k


def test_graph_replayed_backward_is_replay_invariant():
    """A captured minibatch forward+backward gives the eager gradient on every replay (with HIP
    graph packet capture on, the first hidden-layer bias gradient drifted from a later replay on;
    isaacgymenv_amd/__init__.py turns it off)."""
    import isaacgymenv_amd
    assert isaacgymenv_amd.GRAPHS_SAFE
    agent = _agent("Cartpole", 512)
    agent.use_graphs = False
    agent.train_epoch()
    agent.model.train()
    agent.model.running_mean_std.eval()  # frozen input statistics: every call sees the same batch
    agent._mb_forward_backward(0)
    torch.cuda.synchronize()
    ref = agent.flat_grad.clone()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, pool=torch.cuda.graph_pool_handle()):
        agent._mb_forward_backward(0)
    for _ in range(4):
        g.replay()
        torch.cuda.synchronize()
        torch.testing.assert_close(agent.flat_grad, ref, rtol=1e-5, atol=1e-6)


def test_split_k_linear_matches_torch_linear():
    """rl.network.Linear's split-K weight gradient equals nn.Linear's (fp32: 1e-5; fp16 autocast: the
    half-precision rounding of the partial sums, 2e-3 of the gradient's scale)."""
    from isaacgymenv_amd.rl.network import Linear
    torch.manual_seed(0)
    for autocast, direct in ((False, False), (True, False), (False, True), (True, True)):
        lin = Linear(188, 512).cuda()
        lin.direct_grad = direct
        ref = torch.nn.Linear(188, 512).cuda()
        ref.load_state_dict(lin.state_dict())
        x = torch.randn(16384, 188, device="cuda")
        g = torch.randn(16384, 512, device="cuda")
        outs = []
        for m in (lin, ref):
            m.zero_grad()
            xi = x.clone().requires_grad_(True)
            with torch.autocast("cuda", dtype=torch.float16, enabled=autocast):
                y = m(xi)
            (y.float() * g).sum().backward()
            outs.append((y.float(), m.weight.grad.clone(), m.bias.grad.clone(), xi.grad.clone()))
        for a, b in zip(outs[0], outs[1]):
            tol = 2e-3 if autocast else 1e-5
            assert float((a - b).abs().max()) <= tol * float(b.abs().max()) + 1e-6


def test_split_k_linear_autograd_grad_returns_gradients():
    """Outside the learner (direct_grad False), torch.autograd.grad receives the split-K weight and bias
    gradients as results and nothing leaks into .grad."""
    from isaacgymenv_amd.rl.network import Linear
    torch.manual_seed(1)
    lin = Linear(188, 512).cuda()
    ref = torch.nn.Linear(188, 512).cuda()
    ref.load_state_dict(lin.state_dict())
    x = torch.randn(16384, 188, device="cuda")
    gw, gb = torch.autograd.grad(lin(x).sum(), (lin.weight, lin.bias))
    rw, rb = torch.autograd.grad(ref(x).sum(), (ref.weight, ref.bias))
    assert lin.weight.grad is None and lin.bias.grad is None
    assert float((gw - rw).abs().max()) <= 1e-5 * float(rw.abs().max()) + 1e-6
    assert float((gb - rb).abs().max()) <= 1e-5 * float(rb.abs().max()) + 1e-6


@pytest.mark.parametrize("n,offset,dtype", [(96256, 0, torch.float16), (1539, 1, torch.float16),
                                            (4096, 3, torch.float32), (128, 0, torch.float32)])
def test_splitk_accum_kernel_bit_exact(n, offset, dtype):
    """rl_splitk_accum: grad += sum_p parts[p] with the partials added in ascending order in fp32, into a
    gradient view at any float offset of a flat buffer (vector and scalar paths), bit-exact vs numpy."""
    from isaacgymenv_amd.rl import gae
    gen = torch.Generator().manual_seed(n + offset)
    parts = torch.randn(16, n, generator=gen).to(dtype)
    flat = torch.randn(n + 8, generator=gen)
    acc = np.zeros(n, dtype=np.float32)
    for p in parts.float().numpy():
        acc = (acc + p).astype(np.float32)
    want = (flat.numpy()[offset:offset + n] + acc).astype(np.float32)
    d_flat = flat.cuda()
    gae.splitk_accum(parts.cuda(), d_flat[offset:offset + n])
    got = d_flat.cpu().numpy()
    assert np.array_equal(got[offset:offset + n], want)
    assert np.array_equal(np.delete(got, np.s_[offset:offset + n]), np.delete(flat.numpy(), np.s_[offset:offset + n]))


@pytest.mark.parametrize("dones_dtype,boot", [(torch.bool, True), (torch.int64, True), (torch.bool, False)])
def test_rollout_post_kernel_matches_torch_bookkeeping(dones_dtype, boot):
    """rl_rollout_post (one kernel after env.step) = the torch statements of _store_post: experience
    rewards, dones and the episode counters bit-exact over 30 steps with ~5 % dones per step; the
    AverageMeters to fp32 rounding (the kernel reduces the masked sums in its own fixed order)."""
    agent = _agent("Cartpole", 4096 - 37, value_bootstrap=boot, minibatch_size=4096 - 37)
    N = agent.num_actors
    gen = torch.Generator(device="cuda").manual_seed(7)
    state = lambda a: [a.dones, a.current_rewards, a.current_lengths, a.game_rewards.state,  # noqa: E731
                       a.game_lengths.state]
    snap = [t.clone() for t in state(agent)]
    fused, ref = [], []
    steps = []
    for n in range(30):
        rew = torch.randn(N, device="cuda", generator=gen)
        dn = torch.rand(N, device="cuda", generator=gen) < 0.05
        to = dn & (torch.rand(N, device="cuda", generator=gen) < 0.5)
        vals = torch.randn(N, 1, device="cuda", generator=gen)
        steps.append((rew, dn.to(dones_dtype), to.to(dones_dtype), {"values": vals}))
    for mode in ("torch", "fused"):
        for t, s0 in zip(state(agent), snap):
            t.copy_(s0)
        agent.t_rewards.zero_()
        for n, (rew, dn, to, res) in enumerate(steps):
            h = n % agent.horizon
            if mode == "fused":
                agent._store_post_fused(h, res["values"][:, 0], rew, dn, to)
            else:
                agent._s_rew.copy_(rew)
                agent._s_dones.copy_(dn)
                agent._s_timeouts.copy_(to)
                agent._has_timeouts = True
                agent._store_post(h, res)
        torch.cuda.synchronize()
        (fused if mode == "fused" else ref).append([t.clone() for t in state(agent)] + [agent.t_rewards.clone()])
    f, r = fused[0], ref[0]
    for k in (0, 1, 2, 5):
        assert torch.equal(f[k], r[k]), k
    for k in (3, 4):
        torch.testing.assert_close(f[k], r[k], rtol=1e-5, atol=1e-6)
    assert float(r[4][1]) > 0  # the meters were updated


def test_fused_rollout_bookkeeping_equals_torch_statements():
    """play_steps with the two bookkeeping kernels (rl_rollout_pre before env.step; rl_rollout_post
    deferred behind the next act forward, bootstrapping from t_values) fills the same experience,
    bit for bit, as the torch statements in their original order (Cartpole, value bootstrap on)."""
    runs = []
    for fused in (False, True):
        torch.manual_seed(0)
        agent = _agent("Cartpole", 512, value_bootstrap=True)
        agent.use_graphs = False
        agent._fused_post = fused
        returns, values = agent.play_steps()
        torch.cuda.synchronize()
        assert agent._pre_ok is (True if fused else None)
        runs.append([t.clone() for t in (agent.b_obs, agent.t_dones, agent.t_values, agent.t_rewards, agent.b_actions,
                                         agent.b_neglogp, agent.b_mu, agent.b_sigma, agent.dones,
                                         agent.current_rewards, agent.current_lengths, returns, values)])
    assert float(runs[0][1].float().sum()) > 0  # some episodes ended inside the rollout
    for k, (a, b) in enumerate(zip(*runs)):
        assert torch.equal(a, b), k


def test_rollout_pre_kernel_matches_torch_experience_copies():
    """rl_rollout_pre (one kernel before env.step) = the seven torch statements of _store_pre, bit-exact,
    for every horizon slot of a ragged env count (4096 - 37 envs, 12 actions, 188-wide obs)."""
    from isaacgymenv_amd.rl import gae
    N, H, O, A = 4096 - 37, 24, 188, 12
    gen = torch.Generator(device="cuda").manual_seed(11)
    mk = lambda *shape: torch.randn(*shape, device="cuda", generator=gen)  # noqa: E731
    bufs = {"b_obs": torch.zeros(N, H, O, device="cuda"), "t_dones": torch.zeros(H, N, dtype=torch.uint8, device="cuda"),
            "t_values": torch.zeros(H, N, device="cuda"), "b_actions": torch.zeros(N, H, A, device="cuda"),
            "b_neglogp": torch.zeros(N, H, device="cuda"), "b_mu": torch.zeros(N, H, A, device="cuda"),
            "b_sigma": torch.zeros(N, H, A, device="cuda")}
    want = {k: v.clone() for k, v in bufs.items()}
    for n in range(H):
        obs, dones = mk(N, O), (torch.rand(N, device="cuda", generator=gen) < 0.3).to(torch.uint8)
        res = {"values": mk(N, 1), "actions": mk(N, A), "neglogpacs": mk(N), "mus": mk(N, A), "sigmas": mk(N, A).exp()}
        args = (obs, dones, res["values"], res["actions"], res["neglogpacs"], res["mus"], res["sigmas"], *bufs.values())
        assert gae.rollout_pre_applies(*args)
        gae.rollout_pre(n, *args)
        want["b_obs"][:, n] = obs
        want["t_dones"][n] = dones
        want["t_values"][n] = res["values"][:, 0]
        want["b_actions"][:, n] = res["actions"]
        want["b_neglogp"][:, n] = res["neglogpacs"]
        want["b_mu"][:, n] = res["mus"]
        want["b_sigma"][:, n] = res["sigmas"]
    torch.cuda.synchronize()
    for k in bufs:
        assert torch.equal(bufs[k], want[k]), k
    # a layout the kernel does not take is refused (the caller then runs the torch statements)
    assert not gae.rollout_pre_applies(obs.t(), *args[1:])


@pytest.mark.parametrize("rows,cols,dtype,offset", [(16384, 512, torch.float16, 0), (16384, 256, torch.float16, 1),
                                                    (1000, 136, torch.float32, 3), (37, 8, torch.float16, 0)])
def test_colsum_accum_kernel(rows, cols, dtype, offset):
    """rl_colsum_accum: grad += g.sum(0) in fp32 into a gradient view at any float offset; the same
    bits on every call (deterministic two-level order), equal to a float64 column sum to fp32 rounding."""
    from isaacgymenv_amd.rl import gae
    gen = torch.Generator().manual_seed(rows + cols)
    g = torch.randn(rows, cols, generator=gen).to(dtype).cuda()
    flat = torch.randn(cols + 8, generator=gen).cuda()
    outs = []
    for _ in range(3):
        d = flat.clone()
        gae.colsum_accum(g, d[offset:offset + cols])
        outs.append(d.cpu())
    assert all(torch.equal(o, outs[0]) for o in outs[1:])
    want = flat.cpu().double()[offset:offset + cols] + g.cpu().double().sum(0)
    torch.testing.assert_close(outs[0][offset:offset + cols].double(), want, rtol=1e-5, atol=1e-3)
    rest = torch.ones(cols + 8, dtype=torch.bool)
    rest[offset:offset + cols] = False
    assert torch.equal(outs[0][rest], flat.cpu()[rest])



def test_checkpoint_round_trip(tmp_path):
    """save / restore of the learner (model, per-parameter Adam state) is bit-identical."""
    a = _agent("Cartpole", 512)
    a.train_epoch()
    path = str(tmp_path / "ckpt.pth")
    a.save(path)
    b = _agent("Cartpole", 512)
    b.restore(path)
    sa, sb = a.optimizer.state_dict()["state"], b.optimizer.state_dict()["state"]
    assert len(sa) == len(a.params) and sa.keys() == sb.keys()
    for i in sa:
        for k in ("exp_avg", "exp_avg_sq", "step"):
            assert torch.equal(sa[i][k], sb[i][k]), (i, k)
    assert torch.equal(a.flat_param, b.flat_param)
    if a._fused_opt:  # the restored moments are the fused step's flat buffers
        assert torch.equal(a.flat_m, b.flat_m) and torch.equal(a.flat_v, b.flat_v)
        assert b.optimizer.state[b.params[0]]["exp_avg"].data_ptr() == b.flat_m.data_ptr()


def test_fused_ppo_loss_matches_torch_loss():
    """The minibatch loss + gradient as one HIP pass (rl_ppo_loss) against the torch statement of the
    same loss on the same minibatch, fp16 autocast as AnymalTerrainPPO.yaml: loss terms to 1e-4, the flat
    gradient (all parameters) within 1e-2 of its scale (fp16 rounding of the two backward orders)."""
    agent = _agent("AnymalTerrain", 1024, minibatch_size=8192, bounds_loss_coef=0.01)
    assert agent._fused_loss and agent.mixed_precision
    agent.use_graphs = False
    agent.train_epoch()
    agent.model.train()
    agent.model.running_mean_std.eval()
    agent.scaler = torch.amp.GradScaler("cuda", init_scale=1024.0)
    res = {}
    assert agent._fused_heads
    for mode in ("torch", "loss", "heads"):  # torch statement; rl_ppo_loss; rl_ppo_heads_loss (heads + loss)
        agent._fused_loss = mode != "torch"
        agent._fused_heads = mode == "heads"
        out = agent._mb_forward_backward(1)
        torch.cuda.synchronize()
        res[mode] = ([float(x) for x in out[:4]], agent.flat_grad.clone(), out[4].float(), out[5].float())
    l0, g0, m0, s0 = res["torch"]
    for mode in ("loss", "heads"):
        l1, g1, m1, s1 = res[mode]
        np.testing.assert_allclose(l1, l0, rtol=1e-4 if mode == "loss" else 1e-3, atol=1e-6)
        if mode == "loss":  # the same torch heads
            assert torch.equal(m0, m1)
        else:  # the fused heads' fp32 dot products in another order: within one fp16 ulp
            assert float((m1 - m0).abs().max()) <= 2e-3 * max(1.0, float(m0.abs().max()))
        if s1.dim() == 1:  # the fused heads path hands over log sigma
            s1 = torch.exp(s1).expand_as(s0)
        assert torch.allclose(s0, s1)
        scale = float(g0.abs().max())
        assert scale > 0 and float((g1 - g0).abs().max()) <= 1e-2 * scale, (mode, float((g1 - g0).abs().max()), scale)


@pytest.mark.parametrize("rows,cols", [(16384, 188), (4096, 188), (1000, 13), (3, 256)])
def test_rms_normalize_kernel_matches_torch(rows, cols):
    """rl_rms_normalize (train-mode moment update + normalisation, then the eval-mode path) against the
    torch statement of RunningMeanStd on the same inputs: float64 running moments to 1e-6 relative (the
    batch moments' reduction order differs), normalised output to 2e-5."""
    from isaacgymenv_amd.rl import gae
    from isaacgymenv_amd.rl.running_mean_std import RunningMeanStd
    gen = torch.Generator().manual_seed(rows + cols)
    ref = RunningMeanStd((cols,)).cuda()
    mine = RunningMeanStd((cols,)).cuda()
    for step in range(3):
        x = (torch.randn(rows, cols, generator=gen) * (1 + 3 * torch.rand(cols, generator=gen))
             + 5 * torch.randn(cols, generator=gen)).cuda()
        ref.train()
        # the torch statement: a non-contiguous view of x takes RunningMeanStd's torch path
        y_ref = RunningMeanStd.forward(ref, x.t().contiguous().t())
        y = gae.rms_normalize(x, mine.running_mean, mine.running_var, mine.count, mine.epsilon, update=True)
        torch.testing.assert_close(mine.running_mean, ref.running_mean, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(mine.running_var, ref.running_var, rtol=1e-5, atol=1e-6)
        assert float(mine.count) == float(ref.count)
        torch.testing.assert_close(y, y_ref, rtol=2e-5, atol=2e-5)
    y_eval = gae.rms_normalize(x, mine.running_mean, mine.running_var, mine.count, mine.epsilon, update=False)
    ref.eval()
    torch.testing.assert_close(y_eval, RunningMeanStd.forward(ref, x.t().contiguous().t()), rtol=2e-5, atol=2e-5)


def test_policy_head_kernel_matches_torch_act_forward():
    """The act forward through rl_policy_head against the torch statement of the same forward (same
    torch normal_ draws): actions, sigmas and values bit-identical, neglogp to 1e-5."""
    agent = _agent("AnymalTerrain", 1024, minibatch_size=8192)
    agent.use_graphs = False
    agent.train_epoch()
    model = agent.model
    model.eval()
    obs = agent.obs["obs"]
    with torch.no_grad():
        torch.manual_seed(3)
        fused = model({"is_train": False, "obs": obs})
        torch.manual_seed(3)
        # the torch statement: a non-contiguous copy of obs takes RunningMeanStd's torch path and a float64
        # obs is not taken by the fused head; instead call the pieces as the torch path does
        net = model.a2c_network
        o = model.norm_obs(obs)
        mu, logstd, value = net(o)
        sigma = torch.exp(logstd)
        act = torch.empty_like(mu).normal_(0.0, 1.0).mul_(sigma).add_(mu)
        nlp = model.neglogp(act, mu, sigma, logstd)
        val = model.denorm_value(value)
    # the heads are rl_act_heads' FMA chains, the torch statement's a library GEMM: f32 rounding apart
    assert torch.equal(fused["sigmas"], sigma)
    for k, ref in (("mus", mu), ("actions", act), ("values", val)):
        torch.testing.assert_close(fused[k], ref, rtol=1e-5, atol=2e-6, msg=k)
    torch.testing.assert_close(fused["neglogpacs"], nlp, rtol=1e-5, atol=1e-5)


def test_fused_opt_step_matches_torch_adam():
    """rl_opt_step (unscale, found-inf, clip_grad_norm_, Adam, GradScaler.update on flat buffers) against the
    torch statement of rl_games' trancate_gradients_and_step on the same parameters, including a step with a
    non-finite gradient (skipped, scale backed off) and a step the norm clip binds."""
    from isaacgymenv_amd.rl import gae
    torch.manual_seed(3)
    sizes = [(512, 188), (512,), (256, 512), (256,), (12, 128), (12,), (1,)]
    n = sum(int(np.prod(s)) for s in sizes)
    flat0 = torch.randn(n, device="cuda") * 0.1
    # torch reference: separate parameter tensors, fused capturable Adam, a manual GradScaler update
    ref = [torch.nn.Parameter(t.clone().view(s)) for t, s in zip(torch.split(flat0, [int(np.prod(s)) for s in sizes]), sizes)]
    lr = torch.tensor(3e-4, device="cuda")
    opt = torch.optim.Adam(ref, lr=lr, eps=1e-8, fused=True, capturable=True)
    scale_ref = torch.tensor(65536.0, device="cuda")
    tracker_ref = 0
    # fused: flat buffers
    p, m, v = flat0.clone(), torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
    step = torch.zeros((), device="cuda")
    scale = torch.tensor(65536.0, device="cuda")
    tracker = torch.zeros((), dtype=torch.int32, device="cuda")
    part = torch.empty(gae.lib().rl_opt_partials_size(), device="cuda")
    hyper = gae.OptHyper(1.0, 0.9, 0.999, 1e-8, 0.0, 0.5, 2.0, 3)
    for it in range(8):
        g = torch.randn(n, device="cuda") * (0.05 if it % 2 else 5.0) * float(scale_ref)  # odd steps: clip inactive
        if it == 4:
            g[123] = float("inf")
        for t, gg in zip(ref, torch.split(g, [t.numel() for t in ref])):
            t.grad = gg.view_as(t).clone()
        inv = 1.0 / float(scale_ref)
        for t in ref:
            t.grad.mul_(inv)
        found = not all(torch.isfinite(t.grad).all() for t in ref)
        if not found:
            torch.nn.utils.clip_grad_norm_(ref, 1.0)
            opt.step()
            tracker_ref += 1
            if tracker_ref == 3:
                scale_ref *= 2.0
                tracker_ref = 0
        else:
            scale_ref *= 0.5
            tracker_ref = 0
        gae.opt_step(p, g, m, v, step, lr, scale, tracker, hyper, part)
        torch.cuda.synchronize()
        assert float(scale) == float(scale_ref) and int(tracker) == tracker_ref, (it, float(scale), float(scale_ref))
        flat_ref = torch.cat([t.detach().reshape(-1) for t in ref])
        torch.testing.assert_close(p, flat_ref, rtol=1e-5, atol=1e-7)
    assert float(step) == 7.0  # the inf step was skipped
    m_ref = torch.cat([opt.state[t]["exp_avg"].reshape(-1) for t in ref])
    v_ref = torch.cat([opt.state[t]["exp_avg_sq"].reshape(-1) for t in ref])
    torch.testing.assert_close(m, m_ref, rtol=1e-5, atol=1e-9)
    torch.testing.assert_close(v, v_ref, rtol=1e-5, atol=1e-12)


@pytest.mark.parametrize("clip,weight_decay", [(0.0, 0.0), (1.0, 1e-2), (0.0, 1e-3)])
def test_fused_opt_step_without_scaler_matches_torch_adam(clip, weight_decay):
    """rl_opt_step without loss scaling (scale / tracker None: configs with mixed_precision False), with and without
    the norm clip (truncate_grads) and with weight decay, against torch Adam + clip_grad_norm_; a non-finite
    gradient is NOT skipped here (torch's optimizer steps without a GradScaler)."""
    from isaacgymenv_amd.rl import gae
    torch.manual_seed(5)
    sizes = [(64, 20), (64,), (8, 64), (8,)]
    n = sum(int(np.prod(s)) for s in sizes)
    flat0 = torch.randn(n, device="cuda") * 0.1
    ref = [torch.nn.Parameter(t.clone().view(s)) for t, s in zip(torch.split(flat0, [int(np.prod(s)) for s in sizes]), sizes)]
    lr = torch.tensor(1e-3, device="cuda")
    opt = torch.optim.Adam(ref, lr=lr, eps=1e-8, weight_decay=weight_decay, fused=True, capturable=True)
    p, m, v = flat0.clone(), torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
    step = torch.zeros((), device="cuda")
    part = torch.empty(gae.lib().rl_opt_partials_size(), device="cuda")
    hyper = gae.OptHyper(clip, 0.9, 0.999, 1e-8, weight_decay, 0.5, 2.0, 2000)
    for it in range(6):
        g = torch.randn(n, device="cuda") * (3.0 if it % 2 else 0.02)
        for t, gg in zip(ref, torch.split(g, [t.numel() for t in ref])):
            t.grad = gg.view_as(t).clone()
        if clip > 0:
            torch.nn.utils.clip_grad_norm_(ref, clip)
        opt.step()
        gae.opt_step(p, g, m, v, step, lr, None, None, hyper, part)
        torch.cuda.synchronize()
        torch.testing.assert_close(p, torch.cat([t.detach().reshape(-1) for t in ref]), rtol=1e-5, atol=1e-7)
    assert float(step) == 6.0
    # a non-finite gradient: torch steps (NaN parameters follow), so does the fused pass
    g = torch.randn(n, device="cuda")
    g[7] = float("nan")
    gae.opt_step(p, g, m, v, step, lr, None, None, hyper, part)
    torch.cuda.synchronize()
    assert float(step) == 7.0 and not bool(torch.isfinite(p).all())


def test_fused_opt_step_scale_growth_stays_finite():
    """GradScaler growth applies only while the grown scale is finite (torch._amp_update_scale_)."""
    from isaacgymenv_amd.rl import gae
    n = 64
    p, m, v = torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
    step = torch.zeros((), device="cuda")
    scale = torch.tensor(3.0e38, device="cuda")
    s0 = float(scale)
    tracker = torch.zeros((), dtype=torch.int32, device="cuda")
    part = torch.empty(gae.lib().rl_opt_partials_size(), device="cuda")
    hyper = gae.OptHyper(0.0, 0.9, 0.999, 1e-8, 0.0, 0.5, 2.0, 1)
    gae.opt_step(p, torch.ones(n, device="cuda"), m, v, step, torch.tensor(1e-3, device="cuda"), scale, tracker, hyper,
                 part)
    torch.cuda.synchronize()
    assert float(scale) == s0 and int(tracker) == 0 and float(step) == 1.0


@pytest.mark.parametrize("M", [256, 16384])
def test_linear_kernels_exact_on_integers(M):
    """rl_linear_fwd / rl_linear_bwd on small integers (and halves), where fp16 operands, f32 accumulation and
    the fp16 outputs are all exact: the results must equal float64 matmuls bit for bit.  Pins the MFMA operand /
    result lane maps, the tile edges (K = 188 is no multiple of the 32-wide reduction step), both tile sizes
    (M = 256: 64-row tiles) and the split row blocks of the weight-gradient partials."""
    from isaacgymenv_amd.rl import gae
    g = torch.Generator(device="cpu").manual_seed(M)
    ri = lambda lo, hi, *shape: torch.randint(lo, hi + 1, shape, generator=g).to(torch.float16).cuda()  # noqa: E731
    # forward, no activation: |y| <= 188 * 9 + 3 < 2048
    x, w, b = ri(-3, 3, M, 188), ri(-3, 3, 512, 188), ri(-3, 3, 512)
    y = torch.empty(M, 512, dtype=torch.float16, device="cuda")
    gae.linear_fwd(x, w, b, False, y)
    ref = x.double() @ w.double().T + b.double()
    assert torch.equal(y.double(), ref)
    # ELU epilogue on the same sums: only the rounding of expm1 to fp16 differs from torch's fp16 ELU
    gae.linear_fwd(x, w, b, True, y)
    torch.testing.assert_close(y.float(), torch.nn.functional.elu(ref).half().float(), rtol=1e-3, atol=1e-3)
    # backward: y in {-0.5, 0.5, 1, 2} (ELU' = 0.5 or 1), dy in {-1, 0, 1}, w in [-2, 2]
    for N, K, want_dx in ((256, 512, True), (512, 188, False)):
        yv = torch.tensor([-0.5, 0.5, 1.0, 2.0], dtype=torch.float16)[torch.randint(0, 4, (M, N), generator=g)].cuda()
        dy, xw, wv = ri(-1, 1, M, N), ri(-3, 3, M, K), ri(-2, 2, N, K)
        dz = dy.double() * torch.where(yv > 0, 1.0, yv.double() + 1.0)
        splits = 8 if M % (8 * 128) == 0 else 2
        wt = torch.empty(K, N, dtype=torch.float16, device="cuda")
        gae.linear_transpose(wv, wt)
        assert torch.equal(wt, wv.T)
        dx = torch.empty(M, K, dtype=torch.float16, device="cuda") if want_dx else None
        wpart = torch.empty(splits, N, K, device="cuda")
        bpart = torch.empty(splits, N, device="cuda")
        gae.linear_bwd(dy, yv, xw, wv if want_dx else None, dx, splits, wpart, bpart)
        rows = M // splits
        if want_dx:
            assert torch.equal(dx.double(), dz @ wv.double())
        for s_ in range(splits):
            blk = slice(s_ * rows, (s_ + 1) * rows)
            assert torch.equal(wpart[s_].double(), dz[blk].T @ xw[blk].double()), s_
            assert torch.equal(bpart[s_].double(), dz[blk].sum(0)), s_
        # the merged layout: each block's bias partials right behind its weight partials
        part = torch.full((splits, N * K + N), float("nan"), device="cuda")
        gae.linear_bwd(dy, yv, xw, None, None, splits, part, part[:, N * K:], pstride=N * K + N)
        assert torch.equal(part[:, :N * K].reshape(splits, N, K), wpart)
        assert torch.equal(part[:, N * K:], bpart)


def test_linear_kernels_reject_untileable_shapes():
    from isaacgymenv_amd.rl import gae
    x = torch.zeros(100, 64, dtype=torch.float16, device="cuda")
    w = torch.zeros(128, 64, dtype=torch.float16, device="cuda")
    with pytest.raises(RuntimeError, match="M % 64"):
        gae.linear_fwd(x, w, None, True, torch.empty(100, 128, dtype=torch.float16, device="cuda"))
    y = torch.zeros(128, 128, dtype=torch.float16, device="cuda")
    with pytest.raises(RuntimeError, match="K % 128"):
        gae.linear_bwd(y, y, torch.zeros(128, 64, dtype=torch.float16, device="cuda"), w, torch.empty(128, 64, dtype=torch.float16,
                       device="cuda"), 1, torch.empty(1, 128, 64, device="cuda"), None)


def _mlp_pair(obs_dim, units):
    from isaacgymenv_amd.rl import network
    mlp = network._mlp(obs_dim, units, "elu").cuda()
    layers, d = [], obs_dim
    for u in units:
        layers += [torch.nn.Linear(d, u), torch.nn.ELU()]
        d = u
    ref = torch.nn.Sequential(*layers).cuda()
    ref.load_state_dict(mlp.state_dict())
    return mlp, ref


@pytest.mark.parametrize("direct", [False, True])
def test_mfma_mlp_matches_torch_fp32_within_fp16_error(direct, monkeypatch):
    """The actor MLP of AnymalTerrainPPO (188 -> 512 -> 256 -> 128, ELU) on 16384 rows under fp16 autocast through
    the rl_linear kernels, against the same network in fp32 torch.  Bar: the output, the input gradient and every
    parameter gradient lie within 2x (+ a floor of 1e-3 of the field's scale) of the error torch's own fp16 autocast
    path makes against that fp32 reference."""
    from isaacgymenv_amd.rl import network
    torch.manual_seed(3)
    mlp, ref = _mlp_pair(188, [512, 256, 128])
    for m in mlp:
        if isinstance(m, network.Linear):
            m.direct_grad = direct
    with torch.no_grad():
        for p_ in mlp.parameters():
            p_.normal_(0.0, 0.08)
    ref.load_state_dict(mlp.state_dict())
    x = torch.randn(16384, 188, device="cuda") * 1.5
    gout = torch.randn(16384, 128, device="cuda")

    def run(model, autocast, fused):
        monkeypatch.setattr(network, "USE_MFMA_LAYERS", fused)
        model.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.float16, enabled=autocast):
            if fused:
                assert model._fused(x)
            y = model(x)
        (y.float() * gout).sum().backward()
        return [y.float()] + [p_.grad.clone() for p_ in model.parameters()]

    want = run(ref, False, False)
    fp16 = run(mlp, True, False)
    got = run(mlp, True, True)
    for i, (g_, t_, w_) in enumerate(zip(got, fp16, want)):
        scale = float(w_.abs().max())
        err, base = float((g_ - w_).abs().max()), float((t_ - w_).abs().max())
        assert err <= 2.0 * base + 1e-3 * scale, (i, err, base, scale)


def test_mfma_mlp_input_gradient_and_autograd_grad():
    """A grad-requiring input of a 128-multiple width gets its gradient through rl_linear_bwd's dX, and
    torch.autograd.grad (direct off) receives the weight / bias gradients without touching .grad."""
    from isaacgymenv_amd.rl import network
    torch.manual_seed(4)
    mlp, ref = _mlp_pair(256, [256, 128])
    x = torch.randn(4096, 256, device="cuda")
    with torch.autocast("cuda", dtype=torch.float16):
        xi = x.clone().requires_grad_(True)
        assert mlp._fused(xi)
        y = mlp(xi)
        got = torch.autograd.grad(y.float().sum(), [xi] + list(mlp.parameters()))
    xr = x.clone().requires_grad_(True)
    want = torch.autograd.grad(ref(xr).sum(), [xr] + list(ref.parameters()))
    assert all(p_.grad is None for p_ in mlp.parameters())
    for g_, w_ in zip(got, want):
        assert float((g_.float() - w_).abs().max()) <= 5e-3 * float(w_.abs().max()) + 1e-4


def test_mfma_mlp_merged_weight_bias_gradient_path(monkeypatch):
    """with direct gradients and each Linear's weight and bias gradients adjacent in ONE flat buffer
    (the learner's layout, a2c_continuous.A2CAgent), _LinearELUFn takes the merged partial buffer and one
    rl_splitk_accum over the span; with separate gradient tensors the two-finish path.  Both are the same fixed-order
    sums of the same partials, so the gradients agree bit for bit."""
    from isaacgymenv_amd.rl import gae, network
    monkeypatch.setattr(network, "USE_MFMA_LAYERS", True)
    torch.manual_seed(5)
    mlp, _ = _mlp_pair(256, [256, 128])
    lins = [m for m in mlp if isinstance(m, network.Linear)]
    for m in lins:
        m.direct_grad = True
    x = torch.randn(8192, 256, device="cuda")
    gout = torch.randn(8192, 128, device="cuda")
    seen = []
    orig = gae.linear_bwd

    def spy(*a, **kw):
        seen.append(kw.get("pstride", 0))
        return orig(*a, **kw)
    monkeypatch.setattr(gae, "linear_bwd", spy)

    def run(flat_layout):
        if flat_layout:  # weight then bias of each layer, back to back in one buffer (as the learner's flat grad)
            n = sum(p_.numel() for p_ in mlp.parameters())
            flat = torch.zeros(n, device="cuda")
            o = 0
            for m in lins:
                for p_ in (m.weight, m.bias):
                    p_.grad = flat[o:o + p_.numel()].view_as(p_)
                    o += p_.numel()
        else:
            for p_ in mlp.parameters():
                p_.grad = None
        seen.clear()
        with torch.autocast("cuda", dtype=torch.float16):
            assert mlp._fused(x)
            y = mlp(x)
        (y.float() * gout).sum().backward()
        return [p_.grad.clone() for p_ in mlp.parameters()], list(seen)

    merged, pstrides_m = run(True)
    separate, pstrides_s = run(False)
    assert pstrides_m and all(s > 0 for s in pstrides_m), pstrides_m  # the merged layout on every layer
    assert pstrides_s and all(s == 0 for s in pstrides_s), pstrides_s
    for a, b in zip(merged, separate):
        assert torch.equal(a, b)


def _flat_net(net, order, grouped):
    """The learner's flat buffers over `order` (A2CAgent): parameters, their fp16 shadow and the gradients as views
    of three flat tensors, direct gradients; grouped: the actor / critic layer spec (network.GroupedMLPSpec)."""
    from isaacgymenv_amd.rl import network
    offs, off = {}, 0
    flat = torch.cat([p.detach().reshape(-1) for p in order])
    for p in order:
        p.data = flat[off:off + p.numel()].view_as(p)
        offs[id(p)] = off
        off += p.numel()
    half = torch.empty(off, dtype=torch.float16, device="cuda")
    grad = torch.zeros(off, device="cuda")
    for p in order:
        p.grad = grad[offs[id(p)]:offs[id(p)] + p.numel()].view_as(p)
    for m in net.modules():
        if isinstance(m, network.Linear):
            m.half_weight = half[offs[id(m.weight)]:offs[id(m.weight)] + m.weight.numel()].view_as(m.weight)
            m.half_bias = half[offs[id(m.bias)]:offs[id(m.bias)] + m.bias.numel()].view_as(m.bias)
            m.direct_grad = True
    net.grouped = (network.GroupedMLPSpec([net.actor_mlp, net.critic_mlp], half, grad, lambda p: offs[id(p)], flat)
                   if grouped else None)
    half.copy_(flat)
    return grad


def test_grouped_mlp_matches_separate_networks_bit_for_bit(monkeypatch):
    """ABI 6: the actor and critic MLPs of AnymalTerrainPPO (188 -> 512 -> 256 -> 128 ELU, separate) as one launch per
    GEMM (network._GroupedMLPFn: layer 0 one GEMM over the stacked weights, layers 1-2 grouped launches, one gradient
    finish per layer) against each network on its own (_LinearELUFn): hidden outputs and every weight / bias gradient
    bit-identical (same tiles, same reduction order, same split row blocks)."""
    import copy
    from isaacgymenv_amd.rl import network
    monkeypatch.setattr(network, "USE_MFMA_LAYERS", True)
    torch.manual_seed(7)
    base = network.ActorCriticNetwork(188, 12, [512, 256, 128], "elu", separate=True).cuda()
    with torch.no_grad():
        for p_ in base.parameters():
            p_.normal_(0.0, 0.08)
    nets = {}
    for grouped in (True, False):
        net = copy.deepcopy(base)
        order = list(net.parameters())
        if grouped:
            head = []
            lins = [[m for m in mlp if isinstance(m, network.Linear)] for mlp in (net.actor_mlp, net.critic_mlp)]
            for la, lc in zip(*lins):
                head += [la.weight, lc.weight, la.bias, lc.bias]
            ids = {id(p_) for p_ in head}
            order = head + [p_ for p_ in order if id(p_) not in ids]
        _flat_net(net, order, grouped)
        nets[grouped] = net
    x = torch.randn(16384, 188, device="cuda")
    ga, gc = torch.randn(16384, 128, device="cuda"), torch.randn(16384, 128, device="cuda")
    outs = {}
    for grouped, net in nets.items():
        launches = []
        if grouped:
            orig = network._GroupedMLPFn.apply
            monkeypatch.setattr(network._GroupedMLPFn, "apply", lambda *a: (launches.append(1), orig(*a))[1])
        with torch.autocast("cuda", dtype=torch.float16):
            assert net.grouped is None or net.grouped.applies(x)
            a_out, c_out = net.hidden(x)
        ((a_out.float() * ga).sum() + (c_out.float() * gc).sum()).backward()
        assert bool(launches) == grouped
        outs[grouped] = (a_out.detach().clone(), c_out.detach().clone(),
                         {n: p_.grad.clone() for n, p_ in net.named_parameters() if "mlp" in n})
    for a, b in zip(outs[True][:2], outs[False][:2]):
        assert torch.equal(a, b)
    for n, g in outs[False][2].items():
        assert torch.equal(outs[True][2][n], g), n


@pytest.mark.parametrize("vnorm", [True, False])
def test_act_heads_kernel(vnorm):
    """rl_act_heads: the two heads exact on small-integer data (every FMA exact: equal to the float64
    product whatever the order), on strided hidden rows (the grouped act forward's [N][2H] layout, critic
    columns second); the head statements bit-identical to rl_policy_head given the same mu and value."""
    from isaacgymenv_amd.rl import gae
    from isaacgymenv_amd.rl.running_mean_std import RunningMeanStd
    gen = torch.Generator().manual_seed(9)
    N, H, A = 4096 - 37, 128, 12
    ri = lambda lo, hi, *shape: torch.randint(lo, hi, shape, generator=gen).float()  # noqa: E731
    hid = ri(-4, 5, N, 2 * H).cuda()
    a_out, c_out = hid[:, :H], hid[:, H:]
    w_mu, b_mu, w_v, b_v = ri(-3, 4, A, H).cuda(), ri(-8, 9, A).cuda(), ri(-3, 4, 1, H).cuda(), ri(-8, 9, 1).cuda()
    logstd = (torch.randn(A, generator=gen) * 0.3).cuda()
    noise = torch.randn(N, A, generator=gen).cuda()
    vms = None
    if vnorm:
        vms = RunningMeanStd((1,)).cuda()
        vms.running_mean.fill_(0.25)
        vms.running_var.fill_(4.0)
    assert gae.act_heads_applies(a_out, c_out, w_mu, b_mu, w_v, b_v, logstd)
    mu, actions, sigmas, neglogp, values = gae.act_heads(a_out, c_out, w_mu, b_mu, w_v, b_v, noise, logstd, vms)
    want_mu = a_out.cpu().double() @ w_mu.cpu().double().t() + b_mu.cpu().double()
    want_v = c_out.cpu().double() @ w_v.cpu().double().t() + b_v.cpu().double()
    assert torch.equal(mu.cpu().double(), want_mu)
    ref = gae.policy_head(mu, noise, logstd, want_v.float().cuda().contiguous(), vms)
    for got, exp in zip((actions, sigmas, neglogp, values), ref):
        assert torch.equal(got, exp)


@pytest.mark.parametrize("kstep", ["32", "64"])
def test_linear_f32_kernel_exact_on_integers_and_elu(kstep, monkeypatch):
    """rl_linear_fwd_f32_g (the rollout's f32 act-forward layer): with small-integer data every product and partial
    sum is exact in f32, so the kernel equals the float64 product bit for bit whatever its summation order -- this
    pins the MFMA operand maps, the K tail (188 = 5 x 32 + 28), the grouping strides and the bias; with random data
    the ELU epilogue agrees with torch's f32 addmm + elu to f32 rounding.  Both K-stage widths (RL_F32_KSTEP)."""
    from isaacgymenv_amd.rl import gae
    import torch.nn.functional as F
    monkeypatch.setenv("RL_F32_KSTEP", kstep)
    gen = torch.Generator().manual_seed(5)
    M, K0, N0, N1, G = 256, 188, 128, 64, 2
    ri = lambda lo, hi, *shape: torch.randint(lo, hi, shape, generator=gen).float()  # noqa: E731
    x, w0, b0 = ri(-4, 5, M, K0), ri(-4, 5, G, N0, K0), ri(-8, 9, G, N0)
    w1, b1 = ri(-3, 4, G, N1, N0), ri(-8, 9, G, N1)
    xd, w0d, b0d, w1d, b1d = (t.cuda() for t in (x, w0, b0, w1, b1))
    y0 = torch.empty(M, G * N0, device="cuda")
    gae.linear_fwd_f32(xd, K0, K0, w0d, G * N0, b0d, False, y0, G * N0, M)
    want0 = (x.double() @ w0.reshape(G * N0, K0).double().t() + b0.reshape(-1).double())
    assert torch.equal(y0.cpu().double(), want0)
    y1 = torch.empty(M, G * N1, device="cuda")
    gae.linear_fwd_f32(y0, G * N0, N0, w1d, N1, b1d, False, y1, G * N1, M, groups=G, x_gstride=N0,
                       w_gstride=N1 * N0, b_gstride=N1, y_gstride=N1)
    for g in range(G):
        want1 = want0[:, g * N0:(g + 1) * N0] @ w1[g].double().t() + b1[g].double()
        assert torch.equal(y1[:, g * N1:(g + 1) * N1].cpu().double(), want1), g
    xr = torch.randn(M, K0, generator=gen).cuda()
    wr, br = (torch.randn(G * N0, K0, generator=gen) * 0.1).cuda(), torch.randn(G * N0, generator=gen).cuda()
    ye = torch.empty(M, G * N0, device="cuda")
    gae.linear_fwd_f32(xr, K0, K0, wr, G * N0, br, True, ye, G * N0, M)
    torch.testing.assert_close(ye, F.elu(torch.addmm(br, xr, wr.t())), rtol=1e-5, atol=1e-5)


def test_grouped_act_forward_matches_separate_networks():
    """The rollout's act forward (f32, no autograd, no autocast) under the grouped layout: layer 0 one addmm over the
    stacked actor / critic weights, later layers one baddbmm (GroupedMLPSpec.act_forward) against each torch MLP on
    its own; same f32 GEMMs in a different grouping, so within f32 rounding (1e-5)."""
    import copy
    from isaacgymenv_amd.rl import network
    torch.manual_seed(11)
    base = network.ActorCriticNetwork(188, 12, [512, 256, 128], "elu", separate=True).cuda()
    net = copy.deepcopy(base)
    head = []
    lins = [[m for m in mlp if isinstance(m, network.Linear)] for mlp in (net.actor_mlp, net.critic_mlp)]
    for la, lc in zip(*lins):
        head += [la.weight, lc.weight, la.bias, lc.bias]
    ids = {id(p_) for p_ in head}
    _flat_net(net, head + [p_ for p_ in net.parameters() if id(p_) not in ids], True)
    x = torch.randn(4096, 188, device="cuda")
    with torch.no_grad():
        assert net.grouped.act_applies(x) and net.grouped._mfma_f32_applies(x)
        a_g, c_g = net.hidden(x)
        a_r, c_r = base.actor_mlp(x), base.critic_mlp(x)
        mu_g, logstd_g, v_g = net(x)
        mu_r, logstd_r, v_r = base(x)
    torch.testing.assert_close(a_g, a_r, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(c_g, c_r, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(mu_g, mu_r, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(v_g, v_r, rtol=1e-5, atol=1e-5)
    assert torch.equal(logstd_g, logstd_r)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
        assert not net.grouped.act_applies(x)  # the train forward keeps the fp16 MFMA path


@pytest.mark.parametrize("half,M,A", [(True, 16384, 12), (False, 16384, 12), (True, 1000, 8), (False, 3, 1)])
def test_policy_kl_kernel_matches_torch_policy_kl(half, M, A):
    """rl_policy_kl against the torch statement (A2CAgent._policy_kl, rl_games torch_ext.policy_kl) on the same
    tensors: kl within f32 summation-order error; write_back leaves the dataset rows equal to the new mu / sigma
    (dataset.update_mu_sigma)."""
    from isaacgymenv_amd.rl import gae
    from isaacgymenv_amd.rl.a2c_continuous import A2CAgent
    g = torch.Generator(device="cuda").manual_seed(M + A)
    mu_new = torch.randn(M, A, device="cuda", generator=g).to(torch.float16 if half else torch.float32)
    sig_row = torch.exp(0.3 * torch.randn(A, device="cuda", generator=g))
    mu_old = mu_new.float() + 0.05 * torch.randn(M, A, device="cuda", generator=g)
    sg_old = sig_row.expand(M, -1) * torch.exp(0.02 * torch.randn(M, A, device="cuda", generator=g))
    want = A2CAgent._policy_kl(mu_new, sig_row.expand(M, -1), mu_old, sg_old)
    part = torch.zeros(gae.lib().rl_kl_partials_size(), device="cuda")
    for write_back in (False, True):
        kl = torch.empty((), device="cuda")
        mo, so = mu_old.clone(), sg_old.clone()
        gae.policy_kl(mu_new, sig_row, mo, so, kl, part, write_back=write_back)
        torch.testing.assert_close(kl, want, rtol=2e-5, atol=1e-7)
        if write_back:
            assert torch.equal(mo, mu_new.float()) and torch.equal(so, sig_row.expand(M, -1))
        else:
            assert torch.equal(mo, mu_old) and torch.equal(so, sg_old)
    # a per-row sigma [M, A] (row stride A)
    sg_rows = sig_row.expand(M, -1).contiguous() * 1.01
    kl = torch.empty((), device="cuda")
    gae.policy_kl(mu_new, sg_rows, mu_old.clone(), sg_old.clone(), kl, part, write_back=False)
    torch.testing.assert_close(kl, A2CAgent._policy_kl(mu_new, sg_rows, mu_old, sg_old), rtol=2e-5, atol=1e-7)


def test_adaptive_lr_kernel_matches_torch_scheduler():
    """rl_adaptive_lr against A2CAgent._update_lr + the meters of _mb_finish: lr down above 2 thr, up below thr / 2,
    unchanged between, clamps at 1e-6 / 1e-2, the rank average, the f32 optimizer copy; stats bit-identical."""
    from isaacgymenv_amd.rl import gae
    thr = 0.008
    cases = [(0.5, 3e-4), (0.001, 3e-4), (0.008, 3e-4), (0.5, 1.2e-6), (0.0, 9e-3), (0.0161, 5e-4), (0.0039, 5e-4)]
    for world in (1, 4):
        for kl_v, lr_v in cases:
            kl = torch.tensor(kl_v * world, device="cuda")
            lr = torch.tensor(lr_v, dtype=torch.float64, device="cuda")
            opt_lr = torch.tensor(lr_v, device="cuda")
            stats = torch.tensor([1.0, 2.0, 3.0, 4.0], device="cuda")
            losses = torch.tensor([0.25, 0.5, 0.125], device="cuda")
            gae.adaptive_lr(kl, 1.0 / world, True, thr, lr, opt_lr, stats, losses[0], losses[1], losses[2])
            k = torch.tensor(kl_v * world, device="cuda") / world if world > 1 else torch.tensor(kl_v, device="cuda")
            kd, cur = k.double(), torch.tensor(lr_v, dtype=torch.float64, device="cuda")
            want = torch.where(kd > 2.0 * thr, torch.clamp(cur / 1.5, min=1e-6), cur)
            want = torch.where(kd < 0.5 * thr, torch.clamp(cur * 1.5, max=1e-2), want)
            assert torch.equal(kl, k) and torch.equal(lr, want), (kl_v, lr_v, world)
            assert torch.equal(opt_lr, want.float())
            exp = torch.tensor([1.0, 2.0, 3.0, 4.0], device="cuda") + torch.stack([losses[0], losses[1], k, losses[2]])
            assert torch.equal(stats, exp)
    lr = torch.tensor(3e-4, dtype=torch.float64, device="cuda")
    gae.adaptive_lr(torch.tensor(0.5, device="cuda"), 1.0, False, thr, lr, None, None, None, None, None)
    assert float(lr) == 3e-4  # fixed schedule: lr untouched


def test_fused_heads_loss_matches_torch_heads_and_loss():
    """ABI 6: the mu / value heads + PPO loss as one pass (gae.PpoHeadsLossFn over the grouped MLP's stacked output)
    against the torch heads (autocast fp16 GEMMs) + gae.PpoLossFn on the same AnymalTerrainPPO-shaped network and
    minibatch, backward at a GradScaler-like scale: loss and stats to fp32-summation error, mu within one fp16 ulp,
    every parameter gradient (MLP layers, heads, sigma) within fp16 rounding of the torch path's."""
    import copy
    from isaacgymenv_amd.rl import gae, network
    torch.manual_seed(5)
    base = network.ActorCriticNetwork(188, 12, [512, 256, 128], "elu", separate=True).cuda()
    with torch.no_grad():
        for p_ in base.parameters():
            p_.normal_(0.0, 0.08)
        base.sigma.fill_(-0.3)
    M, A = 16384, 12
    g = torch.Generator(device="cuda").manual_seed(9)
    x = torch.randn(M, 188, device="cuda", generator=g)
    actions = torch.randn(M, A, device="cuda", generator=g)
    old_nlp = 12.0 + torch.randn(M, device="cuda", generator=g)
    adv = torch.randn(M, device="cuda", generator=g)
    old_v = torch.randn(M, 1, device="cuda", generator=g)
    ret = old_v + 0.3 * torch.randn(M, 1, device="cuda", generator=g)
    scale = torch.tensor(4096.0, device="cuda")
    outs = {}
    for fused in (False, True):
        net = copy.deepcopy(base)
        head = []
        lins = [[m for m in mlp if isinstance(m, network.Linear)] for mlp in (net.actor_mlp, net.critic_mlp)]
        for la, lc in zip(*lins):
            head += [la.weight, lc.weight, la.bias, lc.bias]
        ids = {id(p_) for p_ in head}
        grad = _flat_net(net, head + [p_ for p_ in net.parameters() if id(p_) not in ids], True)
        args = (actions, old_nlp, adv, old_v, ret, 0.2, True, 2.0, 0.0, 1e-4)
        if fused:
            with torch.autocast("cuda", dtype=torch.float16):
                st = net.stacked_hidden(x)
            assert st is not None
            loss, stats, mu = gae.PpoHeadsLossFn.apply(st[0], st[1], net.sigma.detach(), *args)
        else:
            with torch.autocast("cuda", dtype=torch.float16):
                a_out, c_out = net.hidden(x)
                values, mu = net.value(c_out), net.mu(a_out)
            loss, stats = gae.PpoLossFn.apply(mu, values, net.sigma, *args)
        (loss * scale).backward()
        outs[fused] = (loss.detach().clone(), stats.clone(), mu.detach().clone(),
                       {n: p_.grad.clone() for n, p_ in net.named_parameters()})
    (l0, s0, m0, g0), (l1, s1, m1, g1) = outs[False], outs[True]
    torch.testing.assert_close(l1, l0, rtol=1e-3, atol=1e-5)
    torch.testing.assert_close(s1, s0, rtol=1e-3, atol=1e-5)
    assert m1.dtype == torch.float16
    assert float((m1.float() - m0.float()).abs().max()) <= 2e-3 * max(1.0, float(m0.float().abs().max()))
    for n, ref in g0.items():
        got = g1[n]
        assert float(ref.abs().max()) > 0, n
        err = float((got - ref).abs().max())
        assert err <= 1e-2 * float(ref.abs().max()) + 1e-6, (n, err, float(ref.abs().max()))


def test_policy_kl_step_matches_separate_launches():
    """rl_policy_kl_step (KL + scheduler + meters in one launch, last workgroup finishes) against rl_policy_kl +
    rl_adaptive_lr: kl, lr, the optimizer lr, the meters and the written-back dataset rows bit-identical; the log-sigma
    row (sigma_is_log) against the exp'd row; repeated launches (the counter resets)."""
    from isaacgymenv_amd.rl import gae
    M, A = 16384, 12
    g = torch.Generator(device="cuda").manual_seed(4)
    mu_new = torch.randn(M, A, device="cuda", generator=g).half()
    logstd = 0.2 * torch.randn(A, device="cuda", generator=g)
    mu_old = mu_new.float() + 0.05 * torch.randn(M, A, device="cuda", generator=g)
    sg_old = torch.exp(logstd).expand(M, -1) * torch.exp(0.02 * torch.randn(M, A, device="cuda", generator=g))
    res = {}
    for fused in (False, True):
        part = torch.zeros(gae.lib().rl_kl_partials_size(), device="cuda")
        lr = torch.tensor(3e-4, dtype=torch.float64, device="cuda")
        opt_lr = torch.tensor(3e-4, device="cuda")
        stats = torch.zeros(4, device="cuda")
        losses = torch.tensor([0.25, 0.5, 0.125], device="cuda")
        mo, so = mu_old.clone(), sg_old.clone()
        kls = []
        for rep in range(3):
            kl = torch.empty((), device="cuda")
            if fused:
                gae.policy_kl(mu_new, logstd, mo, so, kl, part, write_back=rep == 0, sigma_is_log=True,
                              lr_step=(True, 0.008, lr, opt_lr, stats, losses[0], losses[1], losses[2]))
            else:
                gae.policy_kl(mu_new, torch.exp(logstd), mo, so, kl, part, write_back=rep == 0)
                gae.adaptive_lr(kl, 1.0, True, 0.008, lr, opt_lr, stats, losses[0], losses[1], losses[2])
            kls.append(kl.clone())
        res[fused] = (torch.stack(kls), lr.clone(), opt_lr.clone(), stats.clone(), mo, so)
    for a, b in zip(res[False], res[True]):
        assert torch.equal(a, b)


def test_opt_step_h_matches_opt_step_and_writes_the_shadow():
    """rl_opt_step_h (shadow write, finish in the Adam launch's last workgroup) against rl_opt_step over several
    steps incl. a non-finite gradient (skipped, scale backed off) and a growth step: parameters, moments, step, scale,
    tracker bit-identical; the shadow equals the parameters rounded to fp16."""
    from isaacgymenv_amd.rl import gae
    n = 300001
    g = torch.Generator(device="cuda").manual_seed(8)
    p0 = torch.randn(n, device="cuda", generator=g)
    grads = [torch.randn(n, device="cuda", generator=g) * 100.0 for _ in range(5)]
    grads[2][17] = float("inf")
    hyper = gae.OptHyper(1.0, 0.9, 0.999, 1e-8, 0.0, 0.5, 2.0, 2)
    res = {}
    for h in (False, True):
        p, m, v = p0.clone(), torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
        half = torch.zeros(n, dtype=torch.float16, device="cuda")
        step, lr = torch.zeros((), device="cuda"), torch.tensor(3e-4, device="cuda")
        scale, tracker = torch.tensor([128.0], device="cuda"), torch.zeros(1, dtype=torch.int32, device="cuda")
        part = torch.zeros(gae.lib().rl_opt_partials_size(), device="cuda")
        for gr in grads:
            if h:
                gae.opt_step_h(p, half, gr, m, v, step, lr, scale, tracker, hyper, part)
            else:
                gae.opt_step(p, gr, m, v, step, lr, scale, tracker, hyper, part)
        res[h] = (p, m, v, step, scale, tracker, half)
    for a, b in zip(res[False][:6], res[True][:6]):
        assert torch.equal(a, b)
    assert float(res[True][3]) == 4.0 and float(res[True][4]) == 256.0  # grow, skip (back off), grow
    assert torch.equal(res[True][6], res[True][0].half())


def test_splitk_accum_multi_matches_per_layer_finishes():
    """rl_splitk_accum_multi: three layers' partials (incl. an unaligned span, an fp16 job) in one launch against
    rl_splitk_accum per layer -- bit-identical; store mode writes the sums into garbage-filled gradients."""
    from isaacgymenv_amd.rl import gae
    g = torch.Generator(device="cuda").manual_seed(2)
    shapes = [(16, 96256 + 1024), (8, 131072 + 512), (4, 32768 + 257)]
    parts = [torch.randn(P, n, device="cuda", generator=g) for P, n in shapes]
    parts[1] = parts[1].half()
    flat = torch.randn(sum(n for _, n in shapes) + 1, device="cuda", generator=g)
    spans, o = [], 1  # offset 1: the first span is not 16-byte aligned
    for _, n in shapes:
        spans.append((o, n))
        o += n
    ref = flat.clone()
    for pt, (o, n) in zip(parts, spans):
        gae.splitk_accum(pt, ref[o:o + n])
    got = flat.clone()
    gae.splitk_accum_multi([(pt, got[o:o + n]) for pt, (o, n) in zip(parts, spans)])
    assert torch.equal(got, ref)
    stored = torch.full_like(flat, float("nan"))
    gae.splitk_accum_multi([(pt, stored[o:o + n]) for pt, (o, n) in zip(parts, spans)], store=True)
    zero = torch.zeros_like(flat)
    for pt, (o, n) in zip(parts, spans):
        gae.splitk_accum(pt, zero[o:o + n])
    assert torch.equal(stored[1:], zero[1:])


def test_rms_normalize_half_output_is_the_rounded_f32_output():
    """rl_rms_normalize_h: the same normalisation (and running-moment update) as rl_rms_normalize, y rounded to fp16."""
    from isaacgymenv_amd.rl import gae
    x = torch.randn(16384, 188, device="cuda") * 3.0 + 1.0
    outs = []
    for half in (False, True):
        mean = torch.zeros(188, dtype=torch.float64, device="cuda")
        var = torch.ones(188, dtype=torch.float64, device="cuda")
        count = torch.tensor(1e-4, dtype=torch.float64, device="cuda")
        y = gae.rms_normalize(x, mean, var, count, 1e-5, True, out_half=half)
        outs.append((y, mean, var, count))
    (y0, *m0), (y1, *m1) = outs
    assert y1.dtype == torch.float16 and torch.equal(y1, y0.half())
    for a, b in zip(m0, m1):
        assert torch.equal(a, b)


@pytest.mark.parametrize("over", [{"units": [512, 512], "minibatch_size": 3072}, {"minibatch_size": 192}])
def test_learner_outside_the_fused_heads_shapes_trains(over):
    """the fused heads + loss pass only where its kernels tile the shapes (minibatch rows a multiple of
    128, last hidden width 32 / 64 / 128 / 256); a [512, 512] MLP or a 192-row minibatch takes the grouped MLPs +
    PpoLossFn path instead of failing at the first minibatch."""
    agent = _agent("AnymalTerrain", 512, **over)
    assert not agent._fused_heads
    agent.env_reset()
    for _ in range(2):
        agent.train_epoch()
    torch.cuda.synchronize()
    assert torch.isfinite(agent.flat_param).all()


def test_fused_heads_minibatch_writes_every_gradient():
    """the fused heads path never zeroes the flat gradient (every element has exactly one writer,
    A2CAgent._grad_store_covers_all): poison the buffer with NaN before one minibatch and check that every element
    is overwritten."""
    agent = _agent("AnymalTerrain", 512, minibatch_size=3072)
    assert agent._fused_heads and agent._grad_store_covers_all
    agent.env_reset()
    agent.train_epoch()  # a real dataset in the buffers
    agent.flat_grad.fill_(float("nan"))
    agent._mb_forward_backward(0)
    torch.cuda.synchronize()
    assert torch.isfinite(agent.flat_grad).all(), int((~torch.isfinite(agent.flat_grad)).sum())
