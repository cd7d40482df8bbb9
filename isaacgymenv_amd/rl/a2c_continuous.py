"""PPO (rl_games ``a2c_continuous`` A2CAgent, rl-games 1.6.x semantics) over a VecTask.

The reference trains every in-scope task with rl_games (isaacgymenvs/train.py:188-218,
cfg/train/*PPO.yaml); rl_games is an external dependency absent from this image and from
/root/reference, so the learner is restated here from its published algorithm:

* rollout (A2CBase.play_steps): ``horizon_length`` steps of act -> VecTask.step; shaped
  reward = scale * r plus ``gamma * V(s) * time_outs`` (value_bootstrap); dones stored u8;
* GAE (A2CBase.discount_values) + returns + swap_and_flatten01: one HIP kernel (rl/gae.py);
* prepare_dataset: advantages = returns - values; value normalisation (RunningMeanStd updated
  with values then returns); advantage normalisation (mean / (std + 1e-8));
* train_epoch: ``mini_epochs`` x contiguous minibatches (PPODataset does not shuffle), clipped
  surrogate, clipped value loss (``critic_coef`` * 0.5), entropy bonus, bound loss, fp16
  autocast + GradScaler (mixed_precision), gradient norm clipping, Adam(eps 1e-8); the
  minibatch's new mu/sigma replace the dataset's old ones (update_mu_sigma); adaptive LR
  (kl > 2 thr -> lr / 1.5, kl < thr / 2 -> lr * 1.5, clamped to [1e-6, 1e-2]) per minibatch.

MI355X-first differences that do not change the arithmetic:
* multi-GPU: the gradients live in ONE flat buffer (parameters' ``.grad`` are views into it),
  so the per-minibatch data-parallel step is a single in-place RCCL all-reduce of 2.09 MB
  (AnymalTerrain) with no concat/scatter copies -- rl_games concatenates the grads, reduces
  and copies them back (trancate_gradients_and_step); the KL average is a device all-reduce;
* the learning rate lives on the device (fused Adam with a tensor lr) and the adaptive schedule
  is evaluated there, so a training epoch has no host synchronisation (rl_games calls
  ``kl.item()`` after every minibatch);
* experience buffers are stored env-major, so the flattened batch is a view, not a copy.
"""
from __future__ import annotations

import math
import os
import time
from dataclasses import dataclass, field
from typing import Any, Dict, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

import isaacgymenv_amd

from . import gae
from .gae import discount_values
from . import network as network_mod
from .network import ActorCriticNetwork, Linear, ModelA2CContinuousLogStd


@dataclass
class PpoConfig:
    """``train.params.config`` keys (cfg/train/AnymalTerrainPPO.yaml:42-82) + network."""
    name: str = "run"
    gamma: float = 0.99
    tau: float = 0.95
    e_clip: float = 0.2
    entropy_coef: float = 0.0
    learning_rate: float = 3e-4
    lr_schedule: Optional[str] = "adaptive"
    kl_threshold: float = 0.008
    truncate_grads: bool = True
    grad_norm: float = 1.0
    horizon_length: int = 24
    minibatch_size: int = 16384
    mini_epochs: int = 5
    critic_coef: float = 2.0
    clip_value: bool = True
    bounds_loss_coef: float = 0.0
    normalize_input: bool = True
    normalize_value: bool = True
    normalize_advantage: bool = True
    value_bootstrap: bool = True
    clip_actions: bool = False
    mixed_precision: bool = True
    reward_scale: float = 1.0
    reward_shift: float = 0.0
    max_epochs: int = 1500
    multi_gpu: bool = False
    weight_decay: float = 0.0
    units: list = field(default_factory=lambda: [512, 256, 128])
    activation: str = "elu"
    separate: bool = True
    fixed_sigma: bool = True
    sigma_init_val: float = 0.0
    games_to_track: int = 100

    @classmethod
    def from_train_cfg(cls, train_cfg: Dict[str, Any], **overrides) -> "PpoConfig":
        """Build from a composed ``train`` config (cfg/train/<Task>PPO.yaml)."""
        p = train_cfg["params"]
        c = dict(p["config"])
        net = p["network"]
        mlp = net.get("mlp", {})
        cont = net.get("space", {}).get("continuous", {})
        shaper = c.get("reward_shaper", {}) or {}
        kw = dict(
            name=str(c.get("name", "run")), gamma=float(c["gamma"]), tau=float(c["tau"]),
            e_clip=float(c["e_clip"]), entropy_coef=float(c.get("entropy_coef", 0.0)),
            learning_rate=float(c["learning_rate"]), lr_schedule=c.get("lr_schedule"),
            kl_threshold=float(c.get("kl_threshold", 0.008)), truncate_grads=bool(c.get("truncate_grads", False)),
            grad_norm=float(c.get("grad_norm", 1.0)), horizon_length=int(c["horizon_length"]),
            minibatch_size=int(c["minibatch_size"]), mini_epochs=int(c["mini_epochs"]),
            critic_coef=float(c.get("critic_coef", 1.0)), clip_value=bool(c.get("clip_value", False)),
            bounds_loss_coef=float(c.get("bounds_loss_coef", 0.0) or 0.0),
            normalize_input=bool(c.get("normalize_input", False)),
            normalize_value=bool(c.get("normalize_value", False)),
            normalize_advantage=bool(c.get("normalize_advantage", True)),
            value_bootstrap=bool(c.get("value_bootstrap", False)), clip_actions=bool(c.get("clip_actions", True)),
            mixed_precision=bool(c.get("mixed_precision", False)),
            reward_scale=float(shaper.get("scale_value", 1.0)), reward_shift=float(shaper.get("shift_value", 0.0)),
            max_epochs=int(c.get("max_epochs", 1500) or 1500), multi_gpu=bool(c.get("multi_gpu", False)),
            weight_decay=float(c.get("weight_decay", 0.0)), units=list(mlp.get("units", [512, 256, 128])),
            activation=str(mlp.get("activation", "elu")), separate=bool(net.get("separate", False)),
            fixed_sigma=bool(cont.get("fixed_sigma", True)),
            sigma_init_val=float((cont.get("sigma_init") or {}).get("val", 0.0)),
        )
        kw.update(overrides)
        return cls(**kw)


class _AverageMeter:
    """rl_games torch_ext.AverageMeter (running mean of the last ``max_size`` finished episodes),
    kept on the device and fed with a done mask so no host sync is needed."""

    def __init__(self, max_size: int, device):
        self.max_size = max_size
        # [mean, current_size] in one buffer (the fused rollout kernel updates both in place)
        self.state = torch.zeros(2, dtype=torch.float32, device=device)
        self.mean = self.state[0]
        self.current_size = self.state[1]

    def update_masked(self, values: torch.Tensor, mask: torch.Tensor):
        cnt = mask.float().sum()
        new_mean = (values * mask).sum() / cnt.clamp(min=1.0)
        size = cnt.clamp(max=float(self.max_size))
        old_size = torch.minimum(self.max_size - size, self.current_size)
        size_sum = old_size + size
        upd = cnt > 0
        # in place: the rollout's captured step graphs hold these tensors
        self.mean.copy_(torch.where(upd, (self.mean * old_size + new_mean * size) / size_sum.clamp(min=1.0), self.mean))
        self.current_size.copy_(torch.where(upd, size_sum, self.current_size))


class A2CAgent:
    """rl_games A2CAgent (continuous) on one rank; ``world_size`` > 1 = data-parallel PPO."""

    def __init__(self, env, cfg: PpoConfig, device: Optional[str] = None, seed: Optional[int] = None,
                 use_graphs: bool = True):
        self.env = env
        self.cfg = cfg
        self.device = torch.device(device or env.rl_device)
        self.num_actors = env.num_envs
        self.obs_dim = env.num_obs
        self.actions_num = env.num_actions
        self.horizon = cfg.horizon_length
        self.batch_size = self.horizon * self.num_actors
        if self.batch_size % cfg.minibatch_size != 0:
            raise ValueError(f"batch {self.batch_size} (horizon x envs) is not divisible by minibatch "
                             f"{cfg.minibatch_size}")
        self.num_minibatches = self.batch_size // cfg.minibatch_size
        self.multi_gpu = cfg.multi_gpu and dist.is_available() and dist.is_initialized() \
            and dist.get_world_size() > 1
        self.rank = dist.get_rank() if self.multi_gpu else 0
        self.world_size = dist.get_world_size() if self.multi_gpu else 1
        if seed is not None:
            torch.manual_seed(seed)
        net = ActorCriticNetwork(self.obs_dim, self.actions_num, cfg.units, cfg.activation, cfg.separate,
                                 cfg.fixed_sigma, cfg.sigma_init_val)
        self.model = ModelA2CContinuousLogStd(net, self.obs_dim, cfg.normalize_input, cfg.normalize_value)
        self.model.to(self.device)
        self.params = [p for p in self.model.parameters()]  # (the optimizer's order: model.parameters())
        self.num_params = sum(p.numel() for p in self.params)
        # the flat layout: model order, except that with separate actor / critic MLPs of equal widths on the fp16
        # matrix-core update, each hidden layer's two weights and then its two biases come first and adjacent, so
        # both networks' layer runs as one launch per GEMM (network.GroupedMLPSpec)
        grouped = (cfg.separate and cfg.mixed_precision and self.device.type == "cuda" and network_mod.USE_MFMA_LAYERS
                   and self._mlps_groupable(net))
        self._flat_params = self.params
        if grouped:
            head = []
            for la, lc in zip(*[[m for m in mlp if isinstance(m, Linear)] for mlp in (net.actor_mlp, net.critic_mlp)]):
                head += [la.weight, lc.weight, la.bias, lc.bias]
            ids = {id(p) for p in head}
            self._flat_params = head + [p for p in self.params if id(p) not in ids]
        # one flat parameter buffer (every parameter a view into it) and, for the fp16 update, its fp16
        # shadow: one cast per minibatch refreshes the fp16 weights every Linear layer reads
        self.flat_param = torch.cat([p.detach().reshape(-1) for p in self._flat_params]).to(self.device)
        offs, off = {}, 0
        for p in self._flat_params:
            p.data = self.flat_param[off:off + p.numel()].view_as(p)
            offs[id(p)] = off
            off += p.numel()
        self.flat_param_half = None
        if cfg.mixed_precision and self.device.type == "cuda":
            self.flat_param_half = torch.empty(self.num_params, dtype=torch.float16, device=self.device)
            for m in self.model.modules():
                if isinstance(m, Linear):
                    o = offs[id(m.weight)]
                    m.half_weight = self.flat_param_half[o:o + m.weight.numel()].view_as(m.weight)
                    if m.bias is not None:
                        o = offs[id(m.bias)]
                        m.half_bias = self.flat_param_half[o:o + m.bias.numel()].view_as(m.bias)
        # one flat gradient buffer; .grad of every parameter is a view into it
        self.flat_grad = torch.zeros(self.num_params, dtype=torch.float32, device=self.device)
        off = 0
        for p in self._flat_params:
            p.grad = self.flat_grad[off:off + p.numel()].view_as(p)
            off += p.numel()
        net.grouped = (network_mod.GroupedMLPSpec([net.actor_mlp, net.critic_mlp], self.flat_param_half, self.flat_grad,
                                                  lambda p: offs[id(p)], self.flat_param) if grouped else None)
        # the learner's .backward() lets the split-K Linear layers accumulate straight into these views
        for m in self.model.modules():
            if isinstance(m, Linear):
                m.direct_grad = True
        if self.multi_gpu:
            self._broadcast_params()
        on_gpu = self.device.type == "cuda"
        self.lr = torch.tensor(cfg.learning_rate, dtype=torch.float64, device=self.device)
        if on_gpu:
            self._opt_lr = torch.tensor(cfg.learning_rate, dtype=torch.float32, device=self.device)
            self.optimizer = torch.optim.Adam(self.params, lr=self._opt_lr, eps=1e-08,
                                              weight_decay=cfg.weight_decay, fused=True, capturable=True)
        else:
            self._opt_lr = None
            self.optimizer = torch.optim.Adam(self.params, lr=cfg.learning_rate, eps=1e-08,
                                              weight_decay=cfg.weight_decay)
        self.mixed_precision = cfg.mixed_precision and on_gpu
        self.scaler = torch.amp.GradScaler("cuda", enabled=self.mixed_precision)
        if self.mixed_precision:  # the scale / growth tracker tensors now (the fused path never calls scale())
            self.scaler._lazy_init_scale_growth_tracker(self.device)
        # the minibatch optimizer step as one HIP pass over the flat buffers (gae.opt_step, rl_opt_step):
        # unscale, found-inf, norm clip, Adam, scaler update -- ~20 launches become 3.  The Adam moments
        # are flat buffers too, and the optimizer's per-parameter state holds views into them, so
        # checkpoints keep torch's Adam state layout.
        self._fused_opt = on_gpu
        if self._fused_opt:
            self.flat_m = torch.zeros_like(self.flat_param)
            self.flat_v = torch.zeros_like(self.flat_param)
            self._opt_step_t = torch.zeros((), dtype=torch.float32, device=self.device)
            self._opt_part = torch.zeros(gae.lib().rl_opt_partials_size(), dtype=torch.float32, device=self.device)
            self._bind_opt_state()
            b1, b2 = self.optimizer.defaults["betas"]
            self._opt_hyper = gae.OptHyper(cfg.grad_norm if cfg.truncate_grads else 0.0, b1, b2,
                                           self.optimizer.defaults["eps"], cfg.weight_decay,
                                           *((self.scaler.get_backoff_factor(), self.scaler.get_growth_factor(),
                                              self.scaler.get_growth_interval()) if self.scaler.is_enabled()
                                             else (0.5, 2.0, 2000)))
        H, N, O, A = self.horizon, self.num_actors, self.obs_dim, self.actions_num
        dev = self.device
        # env-major experience (flattened batch = view); time-major GAE inputs
        self.b_obs = torch.zeros(N, H, O, dtype=torch.float32, device=dev)
        self.b_actions = torch.zeros(N, H, A, dtype=torch.float32, device=dev)
        self.b_neglogp = torch.zeros(N, H, dtype=torch.float32, device=dev)
        self.b_mu = torch.zeros(N, H, A, dtype=torch.float32, device=dev)
        self.b_sigma = torch.zeros(N, H, A, dtype=torch.float32, device=dev)
        self.t_values = torch.zeros(H, N, dtype=torch.float32, device=dev)
        self.t_rewards = torch.zeros(H, N, dtype=torch.float32, device=dev)
        self.t_dones = torch.zeros(H, N, dtype=torch.uint8, device=dev)
        self.current_rewards = torch.zeros(N, dtype=torch.float32, device=dev)
        self.current_lengths = torch.zeros(N, dtype=torch.float32, device=dev)
        self.game_rewards = _AverageMeter(cfg.games_to_track, dev)
        self.game_lengths = _AverageMeter(cfg.games_to_track, dev)
        self.obs = None
        self.dones = torch.zeros(N, dtype=torch.uint8, device=dev)
        self.epoch_num = 0
        self.frame = 0
        self.entropy_coef = cfg.entropy_coef
        self.last_stats: Dict[str, float] = {}
        B = self.batch_size
        self.d_values = torch.zeros(B, 1, dtype=torch.float32, device=dev)
        self.d_returns = torch.zeros(B, 1, dtype=torch.float32, device=dev)
        self.d_adv = torch.zeros(B, dtype=torch.float32, device=dev)
        self.dataset = {
            "old_values": self.d_values, "returns": self.d_returns, "advantages": self.d_adv,
            "old_logp_actions": self.b_neglogp.view(B), "actions": self.b_actions.view(B, -1),
            "obs": self.b_obs.view(B, -1), "mu": self.b_mu.view(B, -1), "sigma": self.b_sigma.view(B, -1),
        }
        self._stats_acc = torch.zeros(4, dtype=torch.float32, device=dev)
        # graphs only with HIP graph packet capture off (isaacgymenv_amd/__init__.py)
        self.use_graphs = on_gpu and use_graphs and isaacgymenv_amd.GRAPHS_SAFE
        self._act_graph = None
        self._g_noise = None
        self._mb_graphs = None
        # rollout bookkeeping around env.step, one (pre, post) graph pair per horizon slot once captured;
        # env outputs are copied into these static buffers first (both paths, same arithmetic)
        self._step_graphs = None
        self._s_rew = torch.zeros(N, dtype=torch.float32, device=dev)
        self._s_dones = torch.zeros(N, dtype=torch.uint8, device=dev)
        self._s_timeouts = torch.zeros(N, dtype=torch.float32, device=dev)
        self._has_timeouts = False
        # after env.step on the GPU: one fused kernel instead of the static copies + post graph
        self._fused_post = on_gpu
        self._pre_ok = None  # rl_rollout_pre fits the experience layouts (decided on first use)
        self._post_checked = False  # rl_rollout_post has checked the agent's own output buffers
        self._t_rew_rows, self._t_val_rows = self.t_rewards.unbind(0), self.t_values.unbind(0)  # per-slot views
        # minibatch loss + gradient as one HIP pass for the fixed-sigma models (every in-scope train
        # config); a learned-sigma head keeps the torch statement of the loss
        net = self.model.a2c_network
        self._fused_loss = on_gpu and net.fixed_sigma and self.actions_num <= 32
        # KL of the minibatch, dataset.update_mu_sigma, adaptive LR and the meters as three HIP launches
        # (gae.policy_kl / gae.adaptive_lr, rl_policy.hip) instead of ~14 torch ones
        self._fused_kl = self._fused_loss and self._opt_lr is not None
        # ... and with the grouped actor / critic layout the heads join the loss pass (network.stacked_hidden)
        # (only where its kernels tile the shapes: every minibatch a multiple of 128 rows -- GroupedMLPSpec.applies --
        # and a last hidden width rl_ppo_heads_loss takes; elsewhere the grouped MLPs + PpoLossFn path runs, decided
        # here because the fused path normalises the input (a running-moments update) before it could fall back)
        self._fused_heads = (self._fused_loss and net.grouped is not None and self.mixed_precision
                             and self.cfg.minibatch_size % 128 == 0
                             and net.mu.in_features in network_mod.HEADS_HIDDEN_SIZES)
        # that path writes every parameter's gradient exactly once (MLP layers, heads, sigma): no zeroing needed
        covered = (sum(p.numel() for p in net.grouped.params) + net.mu.weight.numel() + net.mu.bias.numel()
                   + net.value.weight.numel() + net.value.bias.numel() + net.sigma.numel()) if self._fused_heads else -1
        self._grad_store_covers_all = covered == self.flat_grad.numel()
        # the optimizer writes the fp16 parameter shadow with its update (rl_opt_step_h)
        self._shadow_by_opt = self._fused_opt and self.flat_param_half is not None
        if self._fused_kl:
            self._kl_part = torch.zeros(gae.lib().rl_kl_partials_size(), dtype=torch.float32, device=dev)

    @staticmethod
    def _mlps_groupable(net) -> bool:
        """Actor and critic MLPs of Linear + ELU layers with equal shapes, widths the MFMA kernels tile."""
        if net.critic_mlp is None:
            return False
        mods = [list(net.actor_mlp), list(net.critic_mlp)]
        if len(mods[0]) != len(mods[1]) or not mods[0] or len(mods[0]) % 2:
            return False
        for a, c in zip(*mods):
            if type(a) is not type(c):
                return False
            if isinstance(a, Linear):
                if (a.in_features, a.out_features) != (c.in_features, c.out_features) or a.out_features % 128 \
                        or a.bias is None or c.bias is None:
                    return False
            elif not (type(a) is nn.ELU and a.alpha == 1.0 and c.alpha == 1.0):
                return False
        return True

    # ------------------------------------------------------------------ multi-GPU
    def _broadcast_params(self):
        flat = torch.cat([p.detach().reshape(-1) for p in self._flat_params])
        dist.broadcast(flat, 0)
        off = 0
        with torch.no_grad():
            for p in self._flat_params:
                p.copy_(flat[off:off + p.numel()].view_as(p))
                off += p.numel()

    # ------------------------------------------------------------------ rollout
    _mirror_env = None

    def _obs(self, obs):
        return obs["obs"] if isinstance(obs, dict) else obs

    @torch.no_grad()
    def get_action_values(self, obs):
        """rl_games A2CBase.get_action_values (eval-mode act forward).  After the first epoch on a
        GPU the forward is a replayed HIP graph: the returned tensors are the graph's static outputs,
        valid until the next call."""
        obs = self._obs(obs)
        if self._act_graph is not None:
            # the env's fused tail mirrors each step's observations into the graph's input (amd_set_obs_mirror)
            if obs is not getattr(self._mirror_env, "_obs_mirrored", None) or obs is None:
                self._g_obs.copy_(obs)
            if self._g_noise is not None:  # the act forward's normal_ draws, outside the graph
                self._g_noise.normal_(0.0, 1.0)
            self._act_graph.replay()
            return self._g_res
        self.model.eval()
        return self.model({"is_train": False, "obs": obs})

    @torch.no_grad()
    def get_values(self, obs):
        """rl_games A2CBase.get_values: the full act forward (it samples, consuming RNG)."""
        return self.get_action_values(obs)["values"]

    def env_reset(self):
        self.obs = self.env.reset()
        return self.obs

    def _store_pre(self, n, obs, res):
        """Experience of slot n before env.step (rl_games play_steps' update_data calls)."""
        self.b_obs[:, n] = obs
        self.t_dones[n] = self.dones
        self.t_values[n] = res["values"][:, 0]
        self.b_actions[:, n] = res["actions"]
        self.b_neglogp[:, n] = res["neglogpacs"]
        self.b_mu[:, n] = res["mus"]
        self.b_sigma[:, n] = res["sigmas"]

    def _store_post(self, n, res):
        """After env.step, from the static copies of its outputs: dones, shaped reward (value
        bootstrap on time_outs), episode meters."""
        cfg = self.cfg
        rewards = self._s_rew
        self.dones.copy_(self._s_dones)
        shaped = (rewards + cfg.reward_shift) * cfg.reward_scale
        if cfg.value_bootstrap and self._has_timeouts:
            shaped = shaped + cfg.gamma * res["values"][:, 0] * self._s_timeouts
        self.t_rewards[n] = shaped
        self.current_rewards += rewards
        self.current_lengths += 1
        done = self.dones.bool()
        self.game_rewards.update_masked(self.current_rewards, done)
        self.game_lengths.update_masked(self.current_lengths, done)
        not_done = 1.0 - self.dones.float()
        self.current_rewards *= not_done
        self.current_lengths *= not_done

    def _store_post_fused(self, n, values, rewards, dones, time_outs):
        """_store_post as one HIP kernel (libgymrl rl_rollout_post) reading the env's own output
        buffers: same fp32 arithmetic for the experience rewards, dones and episode counters; the
        meters' masked sums in the kernel's fixed reduction order.  values: slot n's value
        estimates (t_values[n], stored before env.step), for the time-out bootstrap."""
        cfg = self.cfg
        boot = cfg.value_bootstrap and time_outs is not None
        gae.rollout_post(rewards, dones, time_outs if boot else None, values if boot else None,
                         cfg.reward_shift, cfg.reward_scale, cfg.gamma, self.dones, self._t_rew_rows[n],
                         self.current_rewards, self.current_lengths, self.game_rewards.state,
                         self.game_lengths.state, cfg.games_to_track, outputs_checked=self._post_checked)
        self._post_checked = True

    def _store_pre_fused(self, n, obs, res) -> bool:
        """_store_pre as one HIP kernel (libgymrl rl_rollout_pre); False when the layouts do not fit it."""
        args = (obs, self.dones, res["values"], res["actions"], res["neglogpacs"], res["mus"], res["sigmas"],
                self.b_obs, self.t_dones, self.t_values, self.b_actions, self.b_neglogp, self.b_mu, self.b_sigma)
        if self._pre_ok is None:
            self._pre_ok = gae.rollout_pre_applies(*args)
        elif self._pre_ok:  # the act forward's outputs keep their layout; re-check only what varies
            self._pre_ok = obs.is_contiguous() and obs.shape == self.b_obs.shape[::2] and obs.dtype == torch.float32
        if not self._pre_ok:
            return False
        gae.rollout_pre(n, *args)
        return True

    def play_steps(self):
        cfg = self.cfg
        if self.obs is None:
            self.env_reset()
        graphs = self._step_graphs is not None
        # The fused bookkeeping of slot n-1 (rl_rollout_post) is issued after slot n's act forward: it
        # reads only the env's outputs and t_values[n-1], and the forward reads neither, so the GPU gets
        # the forward one host call sooner.  It must precede slot n's experience (which stores dones).
        pending = None
        for n in range(self.horizon):
            res = self.get_action_values(self.obs)
            if pending is not None:
                self._store_post_fused(*pending)
                pending = None
            obs = self._obs(self.obs)
            if not (self._fused_post and self._store_pre_fused(n, obs, res)):
                if graphs:
                    self._step_graphs[n][0].replay()
                else:
                    self._store_pre(n, obs, res)
            actions = res["actions"]
            if cfg.clip_actions:  # action space is [-1, 1]: rescale is identity
                clipped = res.get("actions_clipped")  # (the act graph's static clamp output)
                actions = clipped if clipped is not None else torch.clamp(actions, -1.0, 1.0)
            self.obs, rewards, dones, infos = self.env.step(actions)
            self._has_timeouts = "time_outs" in infos
            if self._fused_post:
                pending = (n, self._t_val_rows[n], rewards, dones, infos.get("time_outs"))
                continue
            self._s_rew.copy_(rewards)
            self._s_dones.copy_(dones)
            if self._has_timeouts:
                self._s_timeouts.copy_(infos["time_outs"])
            if graphs:
                self._step_graphs[n][1].replay()
            else:
                self._store_post(n, res)
        if pending is not None:
            self._store_post_fused(*pending)
        last_values = self.get_values(self.obs)[:, 0].contiguous()
        returns, advs, values = discount_values(self.t_rewards, self.t_values, self.t_dones, last_values,
                                                self.dones.contiguous(), cfg.gamma, cfg.tau)
        self.frame += self.batch_size * self.world_size
        return returns, values

    # ------------------------------------------------------------------ update
    def prepare_dataset(self, returns, values):
        """rl_games A2CBase.prepare_dataset; results land in the persistent dataset buffers."""
        cfg = self.cfg
        advantages = returns - values
        values = values.unsqueeze(1)
        returns = returns.unsqueeze(1)
        if cfg.normalize_value:
            vms = self.model.value_mean_std
            vms.train()
            values = vms(values)
            returns = vms(returns)
            vms.eval()
        if cfg.normalize_advantage:
            advantages = (advantages - advantages.mean()) / (advantages.std() + 1e-8)
        self.d_values.copy_(values)
        self.d_returns.copy_(returns)
        self.d_adv.copy_(advantages)

    def _minibatch(self, i):
        s = slice(i * self.cfg.minibatch_size, (i + 1) * self.cfg.minibatch_size)
        return {k: v[s] for k, v in self.dataset.items()}

    def _mb_forward_backward(self, i):
        """Phase 1 of a minibatch (rl_games calc_gradients up to backward): loss, scaled backward
        into the flat gradient buffer."""
        cfg = self.cfg
        e = cfg.e_clip
        mb = self._minibatch(i)
        if self.mixed_precision and self.flat_param_half is not None and (i == 0 or not self._shadow_by_opt):
            # the fp16 weights of this minibatch, one cast (with rl_opt_step_h the optimizer writes them after each
            # minibatch: only a mini-epoch's first minibatch refreshes them, after whatever changed them outside)
            self.flat_param_half.copy_(self.flat_param)
        if self._fused_loss:
            return self._mb_forward_backward_fused(mb)
        with torch.autocast("cuda", dtype=torch.float16, enabled=self.mixed_precision, cache_enabled=False):
            res = self.model({"is_train": True, "prev_actions": mb["actions"], "obs": mb["obs"]})
            action_log_probs, values, entropy = res["prev_neglogp"], res["values"], res["entropy"]
            mu, sigma = res["mus"], res["sigmas"]
            ratio = torch.exp(mb["old_logp_actions"] - action_log_probs)
            surr1 = mb["advantages"] * ratio
            surr2 = mb["advantages"] * torch.clamp(ratio, 1.0 - e, 1.0 + e)
            a_loss = torch.max(-surr1, -surr2)
            if cfg.clip_value:
                vp_clipped = mb["old_values"] + (values - mb["old_values"]).clamp(-e, e)
                c_loss = torch.max((values - mb["returns"]) ** 2, (vp_clipped - mb["returns"]) ** 2)
            else:
                c_loss = (mb["returns"] - values) ** 2
            soft_bound = 1.1
            b_loss = (torch.clamp_max(mu + soft_bound, 0.0) ** 2 + torch.clamp_min(mu - soft_bound, 0.0) ** 2).sum(-1)
            a_loss, c_loss, entropy, b_loss = a_loss.mean(), c_loss.mean(), entropy.mean(), b_loss.mean()
            loss = a_loss + 0.5 * c_loss * cfg.critic_coef - entropy * self.entropy_coef \
                + b_loss * cfg.bounds_loss_coef
        self.flat_grad.zero_()
        self.scaler.scale(loss).backward()
        return (a_loss.detach(), c_loss.detach(), entropy.detach(), b_loss.detach(), mu.detach(), sigma.detach())

    def _mb_forward_backward_fused(self, mb):
        """_mb_forward_backward with the loss and its gradient as one HIP pass (gae.PpoLossFn,
        rl_ppo_loss): the network forward / backward stay torch + hipBLASLt; the ~80 launches of the
        loss statements and their autograd become three.  Same terms, same autograd rules."""
        cfg = self.cfg
        net = self.model.a2c_network
        if self._fused_heads and self.mixed_precision:
            # the heads and the loss as one pass (gae.PpoHeadsLossFn, rl_ppo_heads_loss) after the grouped MLPs;
            # the normalised obs written as fp16 (the first layer's operand); every gradient stored by its one
            # writer (no zeroing of the flat buffer); the GradScaler scale fed as the loss's gradient (what
            # scaler.scale(loss).backward() computes, minus its two elementwise launches)
            obs_h = self.model.norm_obs_half(mb["obs"])
            with torch.autocast("cuda", dtype=torch.float16, cache_enabled=False):
                st = net.stacked_hidden(obs_h)
            if st is not None:
                y, heads = st
                loss, stats, mu = gae.PpoHeadsLossFn.apply(y, heads, net.sigma.detach(), mb["actions"],
                                                           mb["old_logp_actions"], mb["advantages"], mb["old_values"],
                                                           mb["returns"], cfg.e_clip, cfg.clip_value, cfg.critic_coef,
                                                           self.entropy_coef, cfg.bounds_loss_coef)
                if not self._grad_store_covers_all:
                    self.flat_grad.zero_()
                if self.scaler._scale is None:  # a GradScaler swapped in after construction
                    self.scaler._lazy_init_scale_growth_tracker(self.device)
                torch.autograd.backward(loss, grad_tensors=self.scaler._scale.reshape(()))
                # sigma as the log row (the KL pass takes exp of it)
                return (stats[0], stats[1], stats[2], stats[3], mu, net.sigma.detach())
            raise RuntimeError("fused heads path selected but network.stacked_hidden does not apply")
        obs = self.model.norm_obs(mb["obs"])
        with torch.autocast("cuda", dtype=torch.float16, enabled=self.mixed_precision, cache_enabled=False):
            a_out, c_out = net.hidden(obs)
            values = net.value(c_out)
            mu = net.mu(a_out)
        loss, stats = gae.PpoLossFn.apply(mu, values, net.sigma, mb["actions"], mb["old_logp_actions"],
                                          mb["advantages"], mb["old_values"], mb["returns"], cfg.e_clip,
                                          cfg.clip_value, cfg.critic_coef, self.entropy_coef, cfg.bounds_loss_coef)
        self.flat_grad.zero_()
        self.scaler.scale(loss).backward()
        sigma = torch.exp(net.sigma.detach()).expand(mu.shape[0], -1)
        return (stats[0], stats[1], stats[2], stats[3], mu.detach(), sigma)

    def _bind_opt_state(self):
        """Adam state of every parameter as views into the flat moment buffers (after a checkpoint load
        the loaded tensors are copied in first)."""
        off = 0
        for p in self._flat_params:
            n = p.numel()
            st = self.optimizer.state.get(p)
            m, v = self.flat_m[off:off + n].view_as(p), self.flat_v[off:off + n].view_as(p)
            if st and "exp_avg" in st:
                m.copy_(st["exp_avg"])
                v.copy_(st["exp_avg_sq"])
                self._opt_step_t.copy_(torch.as_tensor(st["step"], dtype=torch.float32))
            self.optimizer.state[p] = {"step": self._opt_step_t, "exp_avg": m, "exp_avg_sq": v}
            off += n

    def _mb_step(self, i, out):
        """Phase 2 (after the gradient all-reduce): unscale, clip, Adam, scaler update; KL of the
        new policy against the dataset's old mu/sigma."""
        if self._fused_opt:
            scale = self.scaler._scale if self.mixed_precision else None
            tracker = self.scaler._growth_tracker if self.mixed_precision else None
            if self._shadow_by_opt:  # + the fp16 shadow of the updated parameters, 2 launches
                gae.opt_step_h(self.flat_param, self.flat_param_half, self.flat_grad, self.flat_m, self.flat_v,
                               self._opt_step_t, self._opt_lr, scale, tracker, self._opt_hyper, self._opt_part)
            else:
                gae.opt_step(self.flat_param, self.flat_grad, self.flat_m, self.flat_v, self._opt_step_t,
                             self._opt_lr, scale, tracker, self._opt_hyper, self._opt_part)
        else:
            if self.cfg.truncate_grads:
                self.scaler.unscale_(self.optimizer)
                nn.utils.clip_grad_norm_(self.params, self.cfg.grad_norm)
            self.scaler.step(self.optimizer)
            self.scaler.update()
        mb = self._minibatch(i)
        with torch.no_grad():
            log_row = out[5].dim() == 1  # the fused heads path hands over log sigma (one row for all)
            if self._fused_kl:  # KL + update_mu_sigma: the dataset rows take the new values in the same pass
                kl = torch.empty((), dtype=torch.float32, device=self.device)
                sig = out[5] if log_row else (out[5][0] if out[5].stride(0) == 0 else out[5])
                # single rank: the scheduler step and the meters in the same launch (no KL all-reduce between)
                lr_step = None if self.multi_gpu else (self.cfg.lr_schedule == "adaptive", self.cfg.kl_threshold,
                                                       self.lr, self._opt_lr, self._stats_acc, out[0], out[1], out[2])
                gae.policy_kl(out[4], sig, mb["mu"], mb["sigma"], kl, self._kl_part, write_back=True,
                              sigma_is_log=log_row, lr_step=lr_step)
                return kl
            sig = torch.exp(out[5]).expand(out[4].shape[0], -1) if log_row else out[5]
            return self._policy_kl(out[4], sig, mb["mu"], mb["sigma"])

    def _mb_finish(self, i, out, kl):
        """Phase 3 (after the KL all-reduce, which sums): dataset.update_mu_sigma, adaptive LR,
        diagnostics."""
        if self._fused_kl:
            if self.multi_gpu:  # (single rank: done in the KL launch, _mb_step)
                gae.adaptive_lr(kl, 1.0 / self.world_size, self.cfg.lr_schedule == "adaptive", self.cfg.kl_threshold,
                                self.lr, self._opt_lr, self._stats_acc, out[0], out[1], out[2])
            return
        s = slice(i * self.cfg.minibatch_size, (i + 1) * self.cfg.minibatch_size)
        with torch.no_grad():
            self.dataset["mu"][s] = out[4]
            self.dataset["sigma"][s] = out[5]
            kl = kl / self.world_size if self.multi_gpu else kl
            self._update_lr(kl)
            self._stats_acc += torch.stack([out[0].float(), out[1].float(), kl.float(), out[2].float()])

    @staticmethod
    def _policy_kl(p0_mu, p0_sigma, p1_mu, p1_sigma):
        c1 = torch.log(p1_sigma / p0_sigma + 1e-5)
        c2 = (p0_sigma ** 2 + (p1_mu - p0_mu) ** 2) / (2.0 * (p1_sigma ** 2 + 1e-5))
        return (c1 + c2 - 0.5).sum(dim=-1).mean()

    def _allreduce_grads(self):
        dist.all_reduce(self.flat_grad, op=dist.ReduceOp.SUM)
        self.flat_grad.div_(self.world_size)

    def calc_gradients(self, mb_index):
        """One minibatch update (rl_games calc_gradients + trancate_gradients_and_step +
        update_mu_sigma + scheduler), eager."""
        out = self._mb_forward_backward(mb_index)
        if self.multi_gpu:
            self._allreduce_grads()
        kl = self._mb_step(mb_index, out)
        if self.multi_gpu:
            dist.all_reduce(kl, op=dist.ReduceOp.SUM)
        self._mb_finish(mb_index, out, kl)
        return out, kl

    def _update_lr(self, kl):
        """AdaptiveScheduler.update on the device (rl_games schedulers.py); ``kl`` is the rank average."""
        if self.cfg.lr_schedule != "adaptive":
            return
        thr = self.cfg.kl_threshold
        kl = kl.double()
        cur = self.lr
        lr = torch.where(kl > 2.0 * thr, torch.clamp(cur / 1.5, min=1e-6), cur)
        lr = torch.where(kl < 0.5 * thr, torch.clamp(cur * 1.5, max=1e-2), lr)
        self.lr.copy_(lr)
        if self._opt_lr is not None:
            self._opt_lr.copy_(lr)
        else:
            for g in self.optimizer.param_groups:
                g["lr"] = float(lr)

    # ------------------------------------------------------------------ HIP graphs
    def _capture_graphs(self):
        """Capture the act forward and every minibatch update as HIP graphs (after one eager epoch
        has initialised optimizer state, scaler and BLAS handles).  Collectives stay outside the
        graphs: with N ranks a minibatch is three graphs around the gradient and KL all-reduces."""
        torch.cuda.synchronize(self.device)
        self.model.eval()
        self._g_obs = torch.zeros(self.num_actors, self.obs_dim, dtype=torch.float32, device=self.device)
        # the sampling noise as a static input drawn before each replay (same normal_ call, same RNG stream):
        # a graph without an RNG node skips torch's two per-replay seed / offset fills
        self._g_noise = torch.zeros(self.num_actors, self.actions_num, dtype=torch.float32, device=self.device)
        self.model.used_input_noise = False
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=torch.cuda.graph_pool_handle()):
            with torch.no_grad():
                self._g_res = self.model({"is_train": False, "obs": self._g_obs, "noise": self._g_noise})
                if self.cfg.clip_actions:  # play_steps' clamp, replayed with the forward (one host launch less)
                    self._g_res["actions_clipped"] = torch.clamp(self._g_res["actions"], -1.0, 1.0)
        if not self.model.used_input_noise:  # the torch statement drew inside the graph
            self._g_noise = None
        self._act_graph = g
        self._mirror_env = None
        env = self.env
        setter = getattr(env, "amd_set_obs_mirror", None)
        if setter is not None and os.environ.get("GS_OBS_MIRROR", "1") != "0" and setter(self._g_obs):
            self._mirror_env = env
        # rollout bookkeeping per horizon slot (reads the act graph's static obs / outputs)
        spool = torch.cuda.graph_pool_handle()
        self._step_graphs = []
        for n in range(self.horizon):
            g_pre, g_post = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.graph(g_pre, pool=spool):
                self._store_pre(n, self._g_obs, self._g_res)
            if not self._fused_post:
                with torch.cuda.graph(g_post, pool=spool):
                    self._store_post(n, self._g_res)
            self._step_graphs.append((g_pre, g_post))
        self.model.train()
        pool = torch.cuda.graph_pool_handle()
        self._mb_graphs = []
        for i in range(self.num_minibatches):
            if not self.multi_gpu:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=pool):
                    out = self._mb_forward_backward(i)
                    kl = self._mb_step(i, out)
                    self._mb_finish(i, out, kl)
                self._mb_graphs.append((g,))
            else:
                g1, g2, g3 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
                with torch.cuda.graph(g1, pool=pool):
                    out = self._mb_forward_backward(i)
                with torch.cuda.graph(g2, pool=pool):
                    self.flat_grad.div_(self.world_size)
                    kl = self._mb_step(i, out)
                with torch.cuda.graph(g3, pool=pool):
                    self._mb_finish(i, out, kl)
                self._mb_graphs.append((g1, g2, g3, kl))
        self.model.eval()
        torch.cuda.synchronize(self.device)

    def _run_minibatch(self, i):
        if self._mb_graphs is None:
            self.calc_gradients(i)
            return
        gs = self._mb_graphs[i]
        if len(gs) == 1:
            gs[0].replay()
            return
        g1, g2, g3, kl = gs
        g1.replay()
        dist.all_reduce(self.flat_grad, op=dist.ReduceOp.SUM)
        g2.replay()
        dist.all_reduce(kl, op=dist.ReduceOp.SUM)
        g3.replay()

    def train_epoch(self):
        t0 = time.perf_counter()
        returns, values = self.play_steps()
        t1 = time.perf_counter()
        self.model.train()
        self.prepare_dataset(returns, values)
        self._stats_acc.zero_()
        for _ in range(self.cfg.mini_epochs):
            for i in range(self.num_minibatches):
                self._run_minibatch(i)
        self.model.eval()
        self.epoch_num += 1
        if self.use_graphs and self._mb_graphs is None:
            self._capture_graphs()
        return t1 - t0

    def epoch_stats(self) -> Dict[str, float]:
        """Host copy of the last epoch's diagnostics (one sync; not called inside the loop)."""
        a, c, kl, ent = (self._stats_acc / (self.cfg.mini_epochs * self.num_minibatches)).tolist()
        return {"epoch": self.epoch_num, "frame": self.frame, "kl": kl, "a_loss": a, "c_loss": c, "entropy": ent,
                "lr": float(self.lr), "mean_reward": float(self.game_rewards.mean),
                "mean_length": float(self.game_lengths.mean)}

    def train(self, max_epochs: Optional[int] = None, log_every: int = 10, printer=print):
        """rl_games ContinuousA2CBase.train loop (no checkpoint cadence); returns the last stats."""
        max_epochs = max_epochs or self.cfg.max_epochs
        stats = {}
        for ep in range(max_epochs):
            t0 = time.perf_counter()
            self.train_epoch()
            if (ep + 1) % log_every == 0 or ep + 1 == max_epochs:
                stats = self.epoch_stats()
                dt = time.perf_counter() - t0
                if self.rank == 0 and printer:
                    printer(f"epoch {stats['epoch']} frames {stats['frame']} fps(last) "
                            f"{self.batch_size * self.world_size / dt:.0f} reward {stats['mean_reward']:.3f} "
                            f"len {stats['mean_length']:.1f} kl {stats['kl']:.4f} lr {stats['lr']:.2e}")
        return stats

    # ------------------------------------------------------------------ checkpoints
    def get_full_state_weights(self):
        return {"model": self.model.state_dict(), "epoch": self.epoch_num, "frame": self.frame,
                "optimizer": self.optimizer.state_dict(), "last_lr": float(self.lr)}

    def save(self, path: str):
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        torch.save(self.get_full_state_weights(), path)

    def restore(self, path: str):
        ckpt = torch.load(path, map_location=self.device, weights_only=True)
        self.model.load_state_dict(ckpt["model"])
        self.epoch_num = int(ckpt.get("epoch", 0))
        self.frame = int(ckpt.get("frame", 0))
        if "optimizer" in ckpt:
            self.optimizer.load_state_dict(ckpt["optimizer"])
            if self._fused_opt:
                self._bind_opt_state()
        lr = float(ckpt.get("last_lr", self.cfg.learning_rate))
        self.lr.fill_(lr)
        if self._opt_lr is not None:
            self._opt_lr.fill_(lr)
