"""rl_games ``actor_critic`` network (network_builder.A2CBuilder, separate=True, fixed sigma)
and the ``continuous_a2c_logstd`` model (models.ModelA2CContinuousLogStd), rl-games 1.6.x.

Train config: isaacgymenvs/cfg/train/AnymalTerrainPPO.yaml:8-30 (mlp 512-256-128 elu,
separate actor/critic, sigma const 0 = std 1, fixed_sigma).  Linear weights keep PyTorch's
default init (rl_games ``default`` initializer = identity), biases are zeroed, as rl_games does.
"""
from __future__ import annotations

import math
import os
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
# The hidden Linear + ELU layers under fp16 autocast (the learner's minibatch forward / backward) run on the matrix
# cores as libgymrl's rl_linear_* kernels (csrc/rl_linear.hip): bias and ELU fused into the GEMM epilogue, ELU's
# backward fused into the dX / dW GEMMs' operand loads.  Off: the torch Linear / ELU statements above.
USE_MFMA_LAYERS = os.environ.get("IGE_MFMA_LAYERS", "1") != "0"  # (an A/B switch for the bench)
# last hidden widths the fused heads + loss kernel takes (rl_ppo_loss.hip heads_check)
HEADS_HIDDEN_SIZES = (32, 64, 128, 256)
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


# the target below (RL_SPLITK_WG, an A/B switch): 128 measured best for AnymalTerrainPPO's grouped layers, whose
# launches run the actor and critic groups side by side (2 x 128 workgroups): update 10.45-10.52 ms per epoch at
# 256, 9.81-9.96 at 128, 11.4 at 64 and 512 (fewer row blocks: fewer f32 partials to write and finish; too few:
# idle CUs) -- profiles/r06x_splitk_sweep.txt
_SPLITK_WG = int(os.environ.get("RL_SPLITK_WG", "128"))


def _splits(M: int, tiles: int) -> int:
    """Row blocks of the weight-gradient partials: enough workgroups to cover the CUs with the layer's 128 x 128
    output tiles (_SPLITK_WG per group), each block a multiple of 128 rows."""
    s = 1
    while s * tiles < _SPLITK_WG and M % (2 * s * 128) == 0:
        s *= 2
    return s


class _LinearELUFn(torch.autograd.Function):
    """One hidden layer, Y = ELU(X W^T + b), on the matrix cores (include/gymrl.h rl_linear_fwd / rl_linear_bwd):
    fp16 operands as torch's autocast would cast them, f32 accumulation, Y rounded once to fp16.  The backward
    takes ELU's derivative from Y (torch's elu_backward on the result), writes dX (fp16) and the weight / bias
    gradients as f32 row-block partials that rl_splitk_accum adds in a fixed order -- into ``.grad`` directly
    under the learner (``direct``, as _SplitKLinearFn), else into fresh tensors autograd returns."""

    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda")
    def forward(ctx, x, w, b, w_half=None, b_half=None, direct=False):
        h = torch.float16
        xc = x.to(h)
        if xc.stride(1) != 1 or xc.stride(0) % 4 or xc.data_ptr() % 8:
            xc = xc.contiguous()
        wc = w_half if w_half is not None else w.to(h)
        bc = None if b is None else (b_half if b_half is not None and w_half is not None else b.to(h))
        y = torch.empty(xc.shape[0], wc.shape[0], dtype=h, device=x.device)
        gae.linear_fwd(xc, wc, bc, True, y)
        ctx.save_for_backward(xc, wc, y)
        ctx.w, ctx.b = w, b
        ctx.direct = bool(direct)
        return y

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, gy):
        xc, wc, y = ctx.saved_tensors
        gy = gy.to(torch.float16).contiguous()
        M, N = y.shape
        K = xc.shape[1]
        dev = y.device
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(M, K, dtype=torch.float16, device=dev)
        want_w = ctx.needs_input_grad[1]
        want_b = ctx.b is not None and ctx.needs_input_grad[2]
        splits = _splits(M, (N // 128) * ((K + 127) // 128))
        gw = gb = None
        w, b = ctx.w, ctx.b
        if ctx.direct and want_w and want_b:
            for p in (w, b):
                if p.grad is None:
                    p.grad = torch.zeros_like(p, dtype=torch.float32)
        # (adjacent views of ONE storage: two separate allocations may also sit back to back, and a span over them
        # would reach past the weight gradient's storage)
        merged = (ctx.direct and want_w and want_b and w.grad.is_contiguous() and b.grad.is_contiguous()
                  and b.grad.untyped_storage().data_ptr() == w.grad.untyped_storage().data_ptr()
                  and b.grad.data_ptr() == w.grad.data_ptr() + 4 * N * K)
        if merged:
            # the learner's flat gradient keeps a Linear's weight and bias adjacent: ONE partial buffer [S][N*K + N]
            # and one finish over both (rl_linear_bwd's merged layout)
            part = torch.empty(splits, N * K + N, dtype=torch.float32, device=dev)
            gae.linear_bwd(gy, y, xc, wc, dx, splits, part, part[:, N * K:], pstride=N * K + N)
            span = w.grad.new_empty(0).set_(w.grad.untyped_storage(), w.grad.storage_offset(), (N * K + N,), (1,))
            gae.splitk_accum(part, span)
            return dx, None, None, None, None, None
        wpart = torch.empty(splits, N, K, dtype=torch.float32, device=dev) if want_w or want_b else None
        bpart = torch.empty(splits, N, dtype=torch.float32, device=dev) if want_b else None
        if dx is not None or wpart is not None:
            gae.linear_bwd(gy, y, xc, wc, dx, splits, wpart, bpart)
        for want, p, part, slot in ((want_w, w, wpart, 0), (want_b, b, bpart, 1)):
            if not want:
                continue
            if ctx.direct:
                if p.grad is None:
                    p.grad = torch.zeros_like(p, dtype=torch.float32)
                gae.splitk_accum(part, p.grad)
            else:
                t = torch.zeros_like(p, dtype=torch.float32)
                gae.splitk_accum(part, t)
                if slot == 0:
                    gw = t
                else:
                    gb = t
        return dx, gw, gb, None, None, None


class GroupedMLPSpec:
    """G equal-shaped Linear + ELU MLPs on one input -- rl_games' separate actor and critic (AnymalTerrainPPO.yaml
    `separate: True`, mlp 512-256-128 elu) -- laid out by the learner (A2CAgent) so that layer l's G weights
    [G][N][K] and then its G biases [G][N] are contiguous in the flat parameter buffer, its fp16 shadow and the flat
    gradient buffer.  _GroupedMLPFn then runs each layer of all G networks as ONE launch per GEMM: layer 0 (one
    shared input) as a single GEMM over the stacked [G*N][K] weight, the later layers as grouped launches
    (include/gymrl.h rl_linear_*_g, ABI 6), and one rl_splitk_accum finishes a layer's G weight and bias gradients."""

    def __init__(self, mlps, flat_half, flat_grad, offset_of, flat_param=None):
        self.G = len(mlps)
        lins = [[m for m in mlp if isinstance(m, Linear)] for mlp in mlps]
        self.params = [p for ls in lins for lin in ls for p in (lin.weight, lin.bias)]
        self.layers, self.layers32 = [], []
        for l, lin0 in enumerate(lins[0]):
            N, K = lin0.out_features, lin0.in_features
            o = offset_of(lin0.weight)
            for g in range(self.G):
                lin = lins[g][l]
                assert (lin.out_features, lin.in_features) == (N, K), "grouped MLPs must have equal shapes"
                assert offset_of(lin.weight) == o + g * N * K and offset_of(lin.bias) == o + self.G * N * K + g * N, \
                    "grouped layout: a layer's G weights, then its G biases"
            G = self.G
            self.layers.append((N, K, flat_half[o:o + G * N * K].view(G * N, K),
                                flat_half[o + G * N * K:o + G * (N * K + N)], flat_grad[o:o + G * (N * K + N)]))
            if flat_param is not None:  # the f32 weights and biases of the layer, [G][N][K] and [G][N]
                self.layers32.append((flat_param[o:o + G * N * K].view(G, N, K),
                                      flat_param[o + G * N * K:o + G * (N * K + N)].view(G, N)))

    def act_forward(self, x):
        """The G MLPs in f32 without autograd (the rollout's act forward, rl_games play_steps: no autocast).  On the
        matrix-core path (rl_linear_fwd_f32_g, include/gymrl.h ABI 7) each layer of all G networks is ONE launch with
        the bias and ELU in its epilogue: layer 0 over the stacked [G*N][K] weight, the later layers grouped, the
        activations [M][G*N] (group g in columns g*N ..).  Otherwise layer 0 is one library GEMM over the stacked
        weights and the later layers one batched GEMM, with one ELU pass per layer.  Returns the G hidden outputs."""
        import torch.nn.functional as F
        G, M = self.G, x.shape[0]
        if self._mfma_f32_applies(x):
            w0, b0 = self.layers32[0]
            n0, k0 = w0.shape[1], w0.shape[2]
            y = torch.empty(M, G * n0, dtype=torch.float32, device=x.device)
            gae.linear_fwd_f32(x, x.stride(0), k0, w0, G * n0, b0, True, y, G * n0, M)
            for w, b in self.layers32[1:]:
                n, k = w.shape[1], w.shape[2]
                z = torch.empty(M, G * n, dtype=torch.float32, device=x.device)
                gae.linear_fwd_f32(y, G * k, k, w, n, b, True, z, G * n, M, groups=G, x_gstride=k, w_gstride=n * k,
                                   b_gstride=n, y_gstride=n)
                y = z
            n = self.layers32[-1][0].shape[1]
            return tuple(y[:, g * n:(g + 1) * n] for g in range(G))
        w0, b0 = self.layers32[0]
        y = torch.addmm(b0.reshape(-1), x, w0.reshape(-1, w0.shape[2]).t())
        F.elu(y, inplace=True)
        y = y.view(M, G, -1).transpose(0, 1)
        for w, b in self.layers32[1:]:
            y = torch.baddbmm(b.unsqueeze(1), y, w.transpose(1, 2))
            F.elu(y, inplace=True)
        return tuple(y[g] for g in range(G))

    def _mfma_f32_applies(self, x) -> bool:
        """The shapes and alignments rl_linear_fwd_f32_g takes (rows % 64, widths % 64, 16-byte rows)."""
        if not USE_MFMA_LAYERS or x.shape[0] % 64 or x.stride(1) != 1 or x.stride(0) % 4 or x.data_ptr() % 16:
            return False
        k_in = x.shape[1]
        for w, b in self.layers32:
            n, k = w.shape[1], w.shape[2]
            if n % 64 or k % 4 or k != k_in or w.data_ptr() % 16 or not (w.is_contiguous() and b.is_contiguous()):
                return False
            k_in = n
        return True

    def act_applies(self, x) -> bool:
        return (bool(self.layers32) and x.is_cuda and x.dtype == torch.float32 and x.dim() == 2
                and not torch.is_grad_enabled() and not torch.is_autocast_enabled("cuda"))

    def applies(self, x) -> bool:
        if not (USE_MFMA_LAYERS and x.is_cuda and x.dim() == 2 and torch.is_autocast_enabled("cuda")
                and torch.get_autocast_dtype("cuda") == torch.float16 and x.shape[0] % 128 == 0 and x.shape[0] > 0):
            return False
        return all(N % 128 == 0 and K % 4 == 0 and (l == 0 or K % 128 == 0) for l, (N, K, *_) in enumerate(self.layers))


class _GroupedMLPFn(torch.autograd.Function):
    """G equal-shaped MLPs (GroupedMLPSpec) forward / backward, one launch per GEMM for all G.  Each group computes
    exactly what _LinearELUFn computes for its network alone (same tiles, same reduction order, same split row
    blocks), so the outputs and gradients are bit-identical to the per-network path
    (tests/test_ppo_gpu.py test_grouped_mlp_matches_separate_networks_bit_for_bit).  The learner's direct
    gradients: the weight and bias gradients go straight into the flat gradient buffer, none is returned."""

    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda")
    def forward(ctx, x, spec, stacked, *params):
        h = torch.float16
        xc = x.to(h)
        if xc.stride(1) != 1 or xc.stride(0) % 4 or xc.data_ptr() % 8:
            xc = xc.contiguous()
        G, M = spec.G, xc.shape[0]
        ys = []
        inp = xc
        for l, (N, K, wh, bh, _) in enumerate(spec.layers):
            y = torch.empty(M, G * N, dtype=h, device=x.device)
            if l == 0:  # one shared input: the stacked [G*N][K] weight is one GEMM
                gae.linear_fwd(xc, wh, bh, True, y)
            else:
                gae.linear_fwd_grouped(inp, G * K, K, wh, N, bh, True, y, G * N, G, K, N * K, N, N, M)
            ys.append(y)
            inp = y
        ctx.save_for_backward(xc, *ys)
        ctx.spec = spec
        ctx.stacked = stacked
        n_last = spec.layers[-1][0]
        if stacked:  # the [M][G*N] output itself (PpoHeadsLossFn reads both groups' columns from it)
            return ys[-1]
        return tuple(ys[-1][:, g * n_last:(g + 1) * n_last] for g in range(G))

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, *gouts):
        xc, *ys = ctx.saved_tensors
        spec = ctx.spec
        G, M = spec.G, xc.shape[0]
        n_last = spec.layers[-1][0]
        if len(gouts) == 1:  # stacked output: the gradient already has the [M][G*N] layout
            dy = gouts[0].to(torch.float16).contiguous()
        else:
            dy = torch.cat([(g if g is not None else torch.zeros(M, n_last, device=xc.device)).to(torch.float16)
                            for g in gouts], dim=1)
        jobs = []
        for l in reversed(range(len(spec.layers))):
            N, K, wh, _, span = spec.layers[l]
            # the per-network path's row blocks (network._LinearELUFn): the same fixed-order partial sums
            splits = _splits(M, (N // 128) * ((K + 127) // 128))
            part = torch.empty(splits, G * (N * K + N), dtype=torch.float32, device=xc.device)
            if l == 0:
                gae.linear_bwd(dy, ys[0], xc, None, None, splits, part, part[:, G * N * K:], pstride=G * (N * K + N))
            else:
                dx = torch.empty(M, G * K, dtype=torch.float16, device=xc.device)
                gae.linear_bwd_grouped(dy, ys[l], G * N, N, M, N, ys[l - 1], G * K, K, K, wh, N * K, dx, G * K, K,
                                       splits, part, part[:, G * N * K:], G * (N * K + N), N * K, N, G)
                dy = dx
            jobs.append((part, span))
        # every layer's weight / bias gradients finished in one launch; the stacked form (the learner's fused heads
        # path, which writes every gradient exactly once) stores them into the unzeroed flat buffer
        gae.splitk_accum_multi(jobs, store=ctx.stacked)
        return (None, None, None) + (None,) * len(spec.params)


class _MLP(nn.Sequential):
    """rl_games' mlp (Linear, activation per hidden layer; same modules and state_dict as nn.Sequential).  Under
    fp16 autocast on the GPU, with ELU layers whose widths the kernels tile (multiples of 128) and a row count in
    multiples of 128, each Linear + ELU pair is one _LinearELUFn."""

    def _fused(self, x) -> bool:
        if not (USE_MFMA_LAYERS and x.is_cuda and x.dim() == 2 and torch.is_autocast_enabled("cuda")
                and torch.get_autocast_dtype("cuda") == torch.float16 and x.shape[0] % 128 == 0 and x.shape[0] > 0):
            return False
        mods = list(self)
        if len(mods) % 2 or not mods:
            return False
        for i in range(0, len(mods), 2):
            lin, act = mods[i], mods[i + 1]
            if not (isinstance(lin, Linear) and type(act) is nn.ELU and act.alpha == 1.0 and not act.inplace
                    and lin.weight.dtype == torch.float32 and lin.out_features % 128 == 0
                    and lin.in_features % 4 == 0):
                return False
            # dX needs the input width in multiples of 128 (every layer after the first: a previous width)
            if i == 0 and x.requires_grad and lin.in_features % 128:
                return False
        return True

    def forward(self, x):
        if not self._fused(x):
            return super().forward(x)
        mods = list(self)
        for i in range(0, len(mods), 2):
            lin = mods[i]
            x = _LinearELUFn.apply(x, lin.weight, lin.bias, lin.half_weight, lin.half_bias, lin.direct_grad)
        return x


def _mlp(in_size: int, units: List[int], activation: str) -> nn.Sequential:
    layers = []
    for u in units:
        layers += [Linear(in_size, u), _ACT[activation]()]
        in_size = u
    return _MLP(*layers)


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

    grouped = None  # GroupedMLPSpec, set by the learner when its flat layout groups the actor and critic layers

    def hidden(self, obs):
        """(actor MLP output, critic MLP output): under the learner's grouped layout one launch per GEMM for both."""
        if self.separate and self.grouped is not None:
            if self.grouped.applies(obs):
                return _GroupedMLPFn.apply(obs, self.grouped, False, *self.grouped.params)
            if self.grouped.act_applies(obs):
                return self.grouped.act_forward(obs)
        a_out = self.actor_mlp(obs)
        return a_out, (self.critic_mlp(obs) if self.separate else a_out)

    def stacked_hidden(self, obs):
        """The grouped actor / critic output as one fp16 [rows][2 * H] tensor (actor columns first) and the heads'
        spec for gae.PpoHeadsLossFn, or None where the grouped MFMA path does not apply (fp16 autocast, learner
        layout, fixed sigma, heads' fp16 shadows and flat gradient views bound).  The backward of this form STORES
        the MLP, head and sigma gradients into their flat-buffer views (each written once): the learner skips
        zeroing the buffer."""
        if not (self.separate and self.fixed_sigma and self.grouped is not None and self.grouped.G == 2
                and self.grouped.applies(obs)):
            return None
        mu, val = self.mu, self.value
        if (mu.half_weight is None or mu.half_bias is None or val.half_weight is None or val.half_bias is None
                or val.out_features != 1 or mu.weight.grad is None or val.weight.grad is None
                or self.sigma.grad is None or mu.in_features % 2):
            return None
        H = mu.in_features
        if H not in HEADS_HIDDEN_SIZES:
            return None
        heads = gae.HeadsSpec(0, H, H, mu.half_weight, mu.half_bias, val.half_weight, val.half_bias, mu.weight.grad,
                              mu.bias.grad, val.weight.grad, val.bias.grad, self.sigma.grad, store=True)
        return _GroupedMLPFn.apply(obs, self.grouped, True, *self.grouped.params), heads

    def forward(self, obs):
        a_out, c_out = self.hidden(obs)
        value = self.value(c_out)
        mu = self.mu(a_out)
        logstd = mu * 0.0 + self.sigma if self.fixed_sigma else self.sigma(a_out)
        return mu, logstd, value


class ModelA2CContinuousLogStd(nn.Module):
    """Input/value normalisation around the network; the act / train forward of rl_games."""

    used_input_noise = False  # set when the act forward took input_dict["noise"] instead of drawing

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

    def norm_obs(self, obs):
        with torch.no_grad():
            return self.running_mean_std(obs) if self.normalize_input else obs

    def norm_obs_half(self, obs):
        """norm_obs rounded to fp16 -- the operand the first fp16 layer casts it to -- written by the normalisation
        pass itself where the device path applies (rl_rms_normalize_h)."""
        with torch.no_grad():
            if self.normalize_input:
                return self.running_mean_std.forward_half(obs)
            return obs.to(torch.float16)

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
            # act forward on the device: the network, torch's normal_ draws, then one kernel for the head
            obs = self.norm_obs(raw)
            a_out, c_out = net.hidden(obs)
            vms = self.value_mean_std if self.normalize_value else None
            heads = (a_out, c_out, net.mu.weight, net.mu.bias, net.value.weight, net.value.bias, net.sigma)
            if USE_MFMA_LAYERS and net.value.out_features == 1 and gae.act_heads_applies(*heads):
                # both heads and the head in one launch (rl_act_heads); the normal_ draws are the same
                # [N, A] call the torch statement makes after mu, so the RNG stream is unchanged.  A caller
                # may pass them drawn already (input_dict["noise"], the act graph's static buffer: the
                # graph then holds no RNG node)
                noise = input_dict.get("noise")
                shape = (a_out.shape[0], net.mu.out_features)
                if noise is not None and noise.shape == shape and noise.dtype == torch.float32 and noise.is_contiguous():
                    self.used_input_noise = True
                else:
                    noise = torch.empty(shape, dtype=torch.float32, device=a_out.device).normal_(0.0, 1.0)
                mu, actions, sigmas, neglogp, values = gae.act_heads(*heads[:6], noise, net.sigma.detach(), vms)
                return {"neglogpacs": neglogp, "values": values, "actions": actions, "mus": mu, "sigmas": sigmas}
            value = net.value(c_out).contiguous()
            mu = net.mu(a_out).contiguous()
            noise = torch.empty_like(mu).normal_(0.0, 1.0)
            actions, sigmas, neglogp, values = gae.policy_head(mu, noise, net.sigma.detach(), value, vms)
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
