"""PPO learner (isaacgymenv_amd/rl) on the CPU: the GAE recurrence against the oracle, the
RunningMeanStd merge, the rl_games loss pieces, a learning run on a toy VecTask-shaped env,
and the data-parallel gradient all-reduce on gloo world_size 2.

rl_games itself is absent (parity unpinned, oracle/ppo_oracle.py header); these tests pin the
restatement to its published formulas."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from isaacgymenv_amd.rl import A2CAgent, PpoConfig
from isaacgymenv_amd.rl.gae import discount_values
from isaacgymenv_amd.rl.running_mean_std import RunningMeanStd
from oracle import ppo_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rollout(H, N, seed, done_p=0.1):
    rng = np.random.RandomState(seed)
    r = rng.randn(H, N).astype(np.float32)
    v = rng.randn(H, N).astype(np.float32)
    d = (rng.rand(H, N) < done_p).astype(np.uint8)
    lv = rng.randn(N).astype(np.float32)
    ld = (rng.rand(N) < done_p).astype(np.uint8)
    return r, v, d, lv, ld


@pytest.mark.parametrize("H,N", [(24, 64), (1, 5), (16, 37)])
def test_gae_torch_path_matches_oracle(H, N):
    r, v, d, lv, ld = _rollout(H, N, seed=H * 100 + N)
    ret, adv, vals = discount_values(*(torch.from_numpy(x) for x in (r, v, d, lv, ld)), 0.99, 0.95)
    oadv = O.discount_values(r, v, d, lv, ld, 0.99, 0.95)
    np.testing.assert_array_equal(adv.numpy(), O.env_major(oadv))
    np.testing.assert_array_equal(ret.numpy(), O.env_major(oadv + v))
    np.testing.assert_array_equal(vals.numpy(), O.env_major(v))


def test_gae_known_answer():
    # one env, no dones: adv_t = sum_k (gamma tau)^k delta_{t+k}
    g, lam = 0.9, 0.5
    r = np.array([[1.0], [0.0], [2.0]], np.float32)
    v = np.array([[0.5], [0.25], [1.0]], np.float32)
    d = np.zeros((3, 1), np.uint8)
    lv, ld = np.array([2.0], np.float32), np.zeros(1, np.uint8)
    delta = [1.0 + g * 0.25 - 0.5, 0.0 + g * 1.0 - 0.25, 2.0 + g * 2.0 - 1.0]
    exp = [delta[0] + g * lam * (delta[1] + g * lam * delta[2]), delta[1] + g * lam * delta[2], delta[2]]
    adv = O.discount_values(r, v, d, lv, ld, g, lam)
    np.testing.assert_allclose(adv[:, 0], exp, rtol=1e-6)
    # a done at t=2 cuts the bootstrap from t=1
    d[2, 0] = 1
    adv = O.discount_values(r, v, d, lv, ld, g, lam)
    assert abs(adv[1, 0] - (0.0 - 0.25)) < 1e-7


def test_running_mean_std_merge():
    rms = RunningMeanStd((3,))
    rms.train()
    m, var, c = np.zeros(3), np.ones(3), 1.0
    rng = np.random.RandomState(0)
    for k in range(4):
        x = (rng.randn(50 + k, 3) * [1, 2, 3] + [1, -1, 0]).astype(np.float32)
        y = rms(torch.from_numpy(x))
        m, var, c = O.rms_merge(m, var, c, x)
        np.testing.assert_allclose(rms.running_mean.numpy(), m, rtol=1e-6)  # batch moments are f32 in torch
        np.testing.assert_allclose(rms.running_var.numpy(), var, rtol=1e-6)
        assert float(rms.count) == c
        exp = np.clip((x - m.astype(np.float32)) / np.sqrt(var.astype(np.float32) + 1e-5), -5, 5)
        np.testing.assert_allclose(y.numpy(), exp, rtol=1e-5, atol=1e-6)
    rms.eval()
    before = rms.running_mean.clone()
    rms(torch.randn(7, 3))
    assert torch.equal(before, rms.running_mean)


class ToyEnv:
    """VecTask-shaped contextual bandit: obs = target in [-0.5,0.5]^2, reward = 1 - |a - target|^2,
    episodes of 4 steps (time_outs on the last), so GAE, bootstrap and resets are exercised."""

    def __init__(self, num_envs=64, seed=0, device="cpu"):
        self.num_envs, self.num_obs, self.num_actions = num_envs, 2, 2
        self.rl_device = device
        self.g = torch.Generator().manual_seed(seed)
        self.target = torch.rand(num_envs, 2, generator=self.g) - 0.5
        self.t = torch.zeros(num_envs, dtype=torch.long)

    def reset(self):
        return {"obs": self.target.clone()}

    def step(self, a):
        rew = 1.0 - ((a - self.target) ** 2).sum(-1)
        self.t += 1
        timeout = self.t >= 4
        done = timeout.clone()
        new = torch.rand(self.num_envs, 2, generator=self.g) - 0.5
        self.target = torch.where(done[:, None], new, self.target)
        self.t = torch.where(done, torch.zeros_like(self.t), self.t)
        return {"obs": self.target.clone()}, rew, done, {"time_outs": timeout}


def _toy_cfg(**kw):
    base = dict(units=[32, 32], horizon_length=8, minibatch_size=128, mini_epochs=4, learning_rate=3e-3,
                entropy_coef=0.0, mixed_precision=False, normalize_input=True, normalize_value=True,
                critic_coef=2.0, kl_threshold=0.016)
    base.update(kw)
    return PpoConfig(**base)


def test_ppo_learns_toy_bandit():
    torch.manual_seed(0)
    env = ToyEnv(64)
    agent = A2CAgent(env, _toy_cfg(), device="cpu", seed=0)
    agent.train_epoch()
    first = agent.epoch_stats()["mean_reward"]
    stats = agent.train(40, printer=None)
    # 4-step episodes: perfect play scores 4, the initial std-1 policy about 4 * (1 - 2 - small)
    assert stats["mean_reward"] > first + 2.0, (first, stats)
    assert np.isfinite(stats["kl"]) and 1e-6 <= stats["lr"] <= 1e-2


def test_ppo_config_from_reference_yaml():
    from isaacgymenv_amd.isaacgymenvs.config import compose
    cfg = compose("config", ["task=AnymalTerrain"])
    p = PpoConfig.from_train_cfg(cfg["train"])
    assert (p.horizon_length, p.minibatch_size, p.mini_epochs, p.units) == (24, 16384, 5, [512, 256, 128])
    assert p.separate and p.fixed_sigma and p.mixed_precision and p.value_bootstrap and p.lr_schedule == "adaptive"
    assert (p.gamma, p.tau, p.e_clip, p.critic_coef, p.entropy_coef) == (0.99, 0.95, 0.2, 2, 0.001)
    # parameter count = the 2,094,692-byte gradient bucket of SURVEY.md 8(e)
    from isaacgymenv_amd.rl.network import ActorCriticNetwork
    net = ActorCriticNetwork(188, 12, p.units, p.activation, p.separate, p.fixed_sigma, p.sigma_init_val)
    assert sum(x.numel() for x in net.parameters()) * 4 == 2094692


def test_policy_kl_and_neglogp_formulas():
    from isaacgymenv_amd.rl.network import ModelA2CContinuousLogStd
    mu0, s0 = torch.randn(5, 3), torch.rand(5, 3) + 0.5
    mu1, s1 = torch.randn(5, 3), torch.rand(5, 3) + 0.5
    kl = A2CAgent._policy_kl(mu0, s0, mu1, s1)
    ref = torch.distributions.kl_divergence(torch.distributions.Normal(mu0, s0),
                                            torch.distributions.Normal(mu1, s1)).sum(-1).mean()
    assert abs(float(kl) - float(ref)) < 1e-3  # rl_games adds 1e-5 regularisers
    x = torch.randn(5, 3)
    nlp = ModelA2CContinuousLogStd.neglogp(x, mu0, s0, torch.log(s0))
    ref = -torch.distributions.Normal(mu0, s0).log_prob(x).sum(-1)
    torch.testing.assert_close(nlp, ref, rtol=1e-5, atol=1e-5)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dp_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(100 + rank)  # different init per rank: the broadcast must make them equal
    env = ToyEnv(32, seed=rank)
    agent = A2CAgent(env, _toy_cfg(multi_gpu=True, minibatch_size=64, lr_schedule=None, truncate_grads=False), device="cpu")
    agent.model.train()
    _load_mb(agent, _dp_batch(rank))
    agent.calc_gradients(0)
    flat = torch.cat([p.detach().reshape(-1) for p in agent.params])
    q.put((rank, flat.numpy(), agent.flat_grad.numpy().copy()))
    dist.destroy_process_group()


def _dp_batch(rank, n=64):
    g = torch.Generator().manual_seed(7 + rank)
    return {"obs": torch.rand(n, 2, generator=g), "actions": torch.randn(n, 2, generator=g),
            "old_logp_actions": torch.rand(n, generator=g) + 1.0, "advantages": torch.randn(n, generator=g),
            "old_values": torch.randn(n, 1, generator=g), "returns": torch.randn(n, 1, generator=g),
            "mu": torch.zeros(n, 2), "sigma": torch.ones(n, 2)}


def test_data_parallel_allreduce_gloo_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dp_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict((r, (w, g)) for r, w, g in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    # identical parameters after the update (broadcast at init + averaged gradients)
    np.testing.assert_array_equal(out[0][0], out[1][0])
    np.testing.assert_array_equal(out[0][1], out[1][1])
    # the averaged gradient equals a single process's gradient on the two minibatches' mean loss
    torch.manual_seed(100)  # rank 0's init = the broadcast parameters
    single = A2CAgent(ToyEnv(32), _toy_cfg(minibatch_size=64, lr_schedule=None, truncate_grads=False), device="cpu")
    single.model.train()
    grads = [_grad_only(single, _dp_batch(r)) for r in range(world)]
    np.testing.assert_allclose(out[0][1], (grads[0] + grads[1]) / 2, rtol=2e-4, atol=1e-6)


def _load_mb(agent, mb):
    n = len(mb["obs"])
    for k, v in mb.items():
        agent.dataset[k][:n] = v


def _grad_only(agent, mb):
    """Gradient of the PPO loss on one minibatch, without stepping (same loss code path)."""
    _load_mb(agent, mb)
    rms_state = {k: v.clone() for k, v in agent.model.running_mean_std.state_dict().items()}
    agent._mb_forward_backward(0)
    agent.model.running_mean_std.load_state_dict(rms_state)
    return agent.flat_grad.numpy().copy()
