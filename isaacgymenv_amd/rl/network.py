"""rl_games ``actor_critic`` network (network_builder.A2CBuilder, separate=True, fixed sigma)
and the ``continuous_a2c_logstd`` model (models.ModelA2CContinuousLogStd), rl-games 1.6.x.

Train config: isaacgymenvs/cfg/train/AnymalTerrainPPO.yaml:8-30 (mlp 512-256-128 elu,
separate actor/critic, sigma const 0 = std 1, fixed_sigma).  Linear weights keep PyTorch's
default init (rl_games ``default`` initializer = identity), biases are zeroed, as rl_games does.
"""
from __future__ import annotations

import math
from typing import Dict, List

import torch
import torch.nn as nn

from . import gae
from .running_mean_std import RunningMeanStd

_ACT = {"elu": nn.ELU, "relu": nn.ReLU, "tanh": nn.Tanh, "selu": nn.SELU, "None": nn.Identity, None: nn.Identity}

# Weight gradients of a minibatch (dW = g^T x, a reduction over the 16384 rows of AnymalTerrainPPO's
# minibatch) are split over SPLIT_K row blocks as one batched GEMM + a float32 sum: as a single GEMM the
# library tiles only the small N x K output (24-48 workgroups for 512 x 188) and takes ~100 us on
# MI355X; split, ~25 us (tools/probes/gemm_splitk.py).  The sum is one HIP kernel that accumulates
# into weight.grad (rl_splitk_accum, csrc/rl_grad.hip).
# the act forward's network as one HIP kernel (gae.act_mlp) instead of the torch Linear / ELU statements.  Off:
# measured 365 us per call against ~0.14 ms for the whole torch act forward (profiles/r03h_kernel_stats.csv): its
# f32 FMA chains wait on L2 weight loads with two waves per SIMD; kept (and parity-tested) as the base for a
# staged-weight version
USE_ACT_KERNEL = False
SPLIT_K = 16
SPLIT_K_MIN_ROWS = 4096


class _SplitKLinearFn(torch.autograd.Function):
    """Linear whose weight gradient is SPLIT_K row-block partial GEMMs finished by ONE HIP kernel that
    adds them (fixed order, fp32) straight into ``weight.grad`` (libgymrl rl_splitk_accum; under the
    learner ``weight.grad`` is a view into its flat gradient buffer).  The forward casts once to the
    autocast dtype and keeps the cast operands for the backward, so the backward re-casts nothing.

    ``direct`` (set by the learner, A2CAgent, whose ``.backward()`` is the only caller) accumulates the weight
    and wide bias gradients straight into ``.grad`` and returns no tensor for them; otherwise (torch.autograd.grad,
    hooks, any other caller) the same kernels finish the sum into a fresh tensor that autograd returns, as
    nn.Linear does."""

    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda")
    def forward(ctx, x, w, b, w_half=None, b_half=None, direct=False):
        dt = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else x.dtype
        # w_half / b_half: the learner's fp16 copies of the parameters, refreshed once per minibatch by
        # one cast of its flat parameter buffer (A2CAgent._refresh_half_params) instead of a cast per tensor
        use_half = w_half is not None and dt == torch.float16
        xc = x.to(dt)
        wc = w_half if use_half else w.to(dt)
        bc = None if b is None else (b_half if use_half and b_half is not None else b.to(dt))
        ctx.save_for_backward(xc, wc)
        ctx.w, ctx.b = w, b
        ctx.has_bias = b is not None
        ctx.direct = bool(direct)
        return torch.nn.functional.linear(xc, wc, bc)

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, g):
        xc, wc = ctx.saved_tensors
        g = g.contiguous()
        gx = g @ wc.to(g.dtype) if ctx.needs_input_grad[0] else None
        gw = None
        if ctx.needs_input_grad[1]:
            w = ctx.w
            rows = g.shape[0]
            parts = torch.bmm(g.reshape(SPLIT_K, rows // SPLIT_K, -1).transpose(1, 2),
                              xc.to(g.dtype).reshape(SPLIT_K, rows // SPLIT_K, -1))
            if ctx.direct:
                if w.grad is None:
                    w.grad = torch.zeros_like(w, dtype=torch.float32)
                gae.splitk_accum(parts, w.grad)
            else:
                gw = torch.zeros_like(w, dtype=torch.float32)
                gae.splitk_accum(parts, gw)
        gb = None
        if ctx.has_bias and ctx.needs_input_grad[2]:
            b = ctx.b
            if gae.colsum_supported(g):
                if ctx.direct:
                    if b.grad is None:
                        b.grad = torch.zeros_like(b, dtype=torch.float32)
                    gae.colsum_accum(g, b.grad)
                else:
                    gb = torch.zeros_like(b, dtype=torch.float32)
                    gae.colsum_accum(g, gb)
            else:  # the narrow heads (value: 1 column, mu: 12)
                gb = g.sum(0, dtype=torch.float32)
        # direct: the weight (and wide bias) gradients are already in .grad (accumulated like autograd would)
        return gx, gw, gb, None, None, None


class Linear(nn.Linear):
    """nn.Linear (same parameters and state_dict) whose backward splits the weight-gradient reduction
    over the batch (SPLIT_K) for the learner's large minibatches."""

    half_weight = None  # fp16 views set by the learner (A2CAgent), else None
    half_bias = None
    direct_grad = False  # set by the learner: its .backward() accumulates straight into .grad

    def forward(self, x):
        if (torch.is_grad_enabled() and x.dim() == 2 and x.shape[0] >= SPLIT_K_MIN_ROWS
                and x.shape[0] % SPLIT_K == 0 and x.is_cuda and self.weight.dtype == torch.float32):
            return _SplitKLinearFn.apply(x, self.weight, self.bias, self.half_weight, self.half_bias, self.direct_grad)
        return super().forward(x)


def _mlp(in_size: int, units: List[int], activation: str) -> nn.Sequential:
    layers = []
    for u in units:
        layers += [Linear(in_size, u), _ACT[activation]()]
        in_size = u
    return nn.Sequential(*layers)


class ActorCriticNetwork(nn.Module):
    def __init__(self, obs_dim: int, actions_num: int, units: List[int], activation: str = "elu",
                 separate: bool = True, fixed_sigma: bool = True, sigma_init_val: float = 0.0, value_size: int = 1):
        super().__init__()
        self.separate = separate
        self.fixed_sigma = fixed_sigma
        self.actor_mlp = _mlp(obs_dim, units, activation)
        self.critic_mlp = _mlp(obs_dim, units, activation) if separate else None
        out = units[-1] if units else obs_dim
        self.value = Linear(out, value_size)
        self.mu = Linear(out, actions_num)
        if fixed_sigma:
            self.sigma = nn.Parameter(torch.zeros(actions_num, dtype=torch.float32), requires_grad=True)
        else:
            self.sigma = Linear(out, actions_num)
        for m in self.modules():
            if isinstance(m, nn.Linear) and m.bias is not None:
                nn.init.zeros_(m.bias)
        with torch.no_grad():  # const_initializer
            if fixed_sigma:
                self.sigma.fill_(sigma_init_val)
            else:
                self.sigma.weight.fill_(sigma_init_val)

    def forward(self, obs):
        a_out = self.actor_mlp(obs)
        c_out = self.critic_mlp(obs) if self.separate else a_out
        value = self.value(c_out)
        mu = self.mu(a_out)
        logstd = mu * 0.0 + self.sigma if self.fixed_sigma else self.sigma(a_out)
        return mu, logstd, value


class ModelA2CContinuousLogStd(nn.Module):
    """Input/value normalisation around the network; the act / train forward of rl_games."""

    def __init__(self, net: ActorCriticNetwork, obs_dim: int, normalize_input: bool = True,
                 normalize_value: bool = True, value_size: int = 1):
        super().__init__()
        self.a2c_network = net
        self.normalize_input = normalize_input
        self.normalize_value = normalize_value
        if normalize_value:
            self.value_mean_std = RunningMeanStd((value_size,))
        if normalize_input:
            self.running_mean_std = RunningMeanStd((obs_dim,))

    def _act_mlps(self):
        """(actor, critic or None) rl_mlp descriptors for gae.act_mlp, or None when the act kernel cannot run this
        model (the parameter pointers are stable: the learner keeps them as views into its flat buffer)."""
        if not USE_ACT_KERNEL:
            return None
        if getattr(self, "_act_desc", None) is None:
            net = self.a2c_network
            a = gae.mlp_desc(net.actor_mlp)
            c = gae.mlp_desc(net.critic_mlp) if net.separate else None
            ok = a is not None and (c is not None or not net.separate) and net.mu.weight.dtype == torch.float32
            if ok and self.normalize_input:
                rms = self.running_mean_std
                ok = rms.running_mean.dtype == torch.float64 and not rms.norm_only
            self._act_desc = (a, c, gae.act_mlp_workspace(a, c, net.mu.weight.device)) if ok else False
        return self._act_desc or None

    def norm_obs(self, obs):
        with torch.no_grad():
            return self.running_mean_std(obs) if self.normalize_input else obs

    def denorm_value(self, value):
        with torch.no_grad():
            return self.value_mean_std(value, unnorm=True) if self.normalize_value else value

    @staticmethod
    def neglogp(x, mean, std, logstd):
        return 0.5 * torch.sum(((x - mean) / std) ** 2, dim=-1) \
            + 0.5 * math.log(2.0 * math.pi) * x.size()[-1] + torch.sum(logstd, dim=-1)

    def forward(self, input_dict: Dict[str, torch.Tensor]):
        is_train = input_dict.get("is_train", True)
        prev_actions = input_dict.get("prev_actions", None)
        raw = input_dict["obs"]
        net = self.a2c_network
        if (not is_train and raw.is_cuda and raw.dtype == torch.float32 and net.fixed_sigma
                and (not self.normalize_value or self.value_mean_std.running_mean.numel() == 1)):
            # act forward on the device: the network (one kernel, gae.act_mlp, when its layers allow it and the input
            # statistics are frozen -- eval mode, as rl_games' play_steps sets), torch's normal_ draws, then one
            # kernel for the head
            frozen = not (self.normalize_input and self.running_mean_std.training)
            mlps = self._act_mlps() if frozen and raw.is_contiguous() else None
            if mlps is not None:
                mu, value = gae.act_mlp(raw, self.running_mean_std if self.normalize_input else None,
                                        mlps[0], mlps[1], net.mu, net.value, mlps[2])
            else:
                obs = self.norm_obs(raw)
                a_out = net.actor_mlp(obs)
                c_out = net.critic_mlp(obs) if net.separate else a_out
                value = net.value(c_out).contiguous()
                mu = net.mu(a_out).contiguous()
            noise = torch.empty_like(mu).normal_(0.0, 1.0)
            actions, sigmas, neglogp, values = gae.policy_head(
                mu, noise, net.sigma.detach(), value, self.value_mean_std if self.normalize_value else None)
            return {"neglogpacs": neglogp, "values": values, "actions": actions, "mus": mu, "sigmas": sigmas}
        obs = self.norm_obs(raw)
        mu, logstd, value = self.a2c_network(obs)
        sigma = torch.exp(logstd)
        distr = torch.distributions.Normal(mu, sigma, validate_args=False)
        if is_train:
            entropy = distr.entropy().sum(dim=-1)
            prev_neglogp = self.neglogp(prev_actions, mu, sigma, logstd)
            return {"prev_neglogp": torch.squeeze(prev_neglogp), "values": value, "entropy": entropy,
                    "mus": mu, "sigmas": sigma}
        # = Normal.sample() = torch.normal(mu, sigma), whose ATen body is normal_(0, 1) * std + mean;
        # spelled out because torch.normal's std >= 0 check syncs the host (not capturable in a graph)
        selected_action = torch.empty_like(mu).normal_(0.0, 1.0).mul_(sigma).add_(mu)
        neglogp = self.neglogp(selected_action, mu, sigma, logstd)
        return {"neglogpacs": torch.squeeze(neglogp), "values": self.denorm_value(value),
                "actions": selected_action, "mus": mu, "sigmas": sigma}
