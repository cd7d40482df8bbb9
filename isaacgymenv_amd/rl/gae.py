"""ctypes binding of libgymrl.so (include/gymrl.h).

``discount_values`` is rl_games ``A2CBase.discount_values`` (a2c_common.py, rl-games 1.6.x)
fused with ``returns = advs + values`` and ``swap_and_flatten01``.  Device tensors go through
the HIP kernel; there is no torch fallback for them (a missing library raises).  Host tensors
(the CPU pipeline, rl_device=cpu) use the torch loop below, which is the reference's own
statement of the recurrence.
"""
from __future__ import annotations

import ctypes as C
import os

import torch
from isaacgymenv_amd._stream import raw_stream

LIB_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_lib", "libgymrl.so")
EXPORTED_SYMBOLS = ["rl_abi_version", "rl_last_error", "rl_gae", "rl_splitk_accum", "rl_colsum_accum", "rl_rollout_post",
                    "rl_ppo_loss", "rl_ppo_loss_backward", "rl_rms_normalize", "rl_opt_step", "rl_opt_partials_size",
                    "rl_linear_fwd", "rl_linear_transpose", "rl_linear_bwd", "rl_policy_head", "rl_linear_fwd_g",
                    "rl_linear_bwd_g", "rl_kl_partials_size", "rl_policy_kl", "rl_adaptive_lr",
                    "rl_ppo_heads_partials_size", "rl_ppo_heads_loss", "rl_ppo_heads_loss_backward",
                    "rl_splitk_accum_multi", "rl_policy_kl_step", "rl_opt_step_h", "rl_rms_normalize_h", "rl_rollout_pre",
                    "rl_linear_fwd_f32_g", "rl_act_heads"]
_lib = None


RL_ABI_VERSION = 7  # include/gymrl.h


class LinearGroups(C.Structure):
    """include/gymrl.h rl_linear_groups"""
    _fields_ = [("groups", C.c_int32), ("ldy", C.c_int32), ("lddx", C.c_int32), ("reserved", C.c_int32),
                ("x_gstride", C.c_int64), ("w_gstride", C.c_int64), ("b_gstride", C.c_int64), ("y_gstride", C.c_int64),
                ("dx_gstride", C.c_int64), ("part_gstride", C.c_int64), ("bpart_gstride", C.c_int64)]


SPLITK_MAX_JOBS = 8  # include/gymrl.h RL_SPLITK_MAX_JOBS


class SplitkJob(C.Structure):
    """include/gymrl.h rl_splitk_job."""
    _fields_ = [("parts", C.c_void_p), ("grad", C.c_void_p), ("n", C.c_int64), ("num_parts", C.c_int32),
                ("parts_are_f16", C.c_int32)]


class OptHyper(C.Structure):
    """include/gymrl.h rl_opt_hyper"""
    _fields_ = [("max_norm", C.c_float), ("beta1", C.c_float), ("beta2", C.c_float), ("eps", C.c_float),
                ("weight_decay", C.c_float), ("backoff", C.c_float), ("growth", C.c_float),
                ("growth_interval", C.c_int32)]


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build it with `python -m isaacgymenv_amd.build`. "
                               "Device tensors have no torch fallback for GAE.")
        L = C.CDLL(LIB_PATH)
        L.rl_abi_version.restype = C.c_int
        got = L.rl_abi_version()
        if got != RL_ABI_VERSION:
            raise RuntimeError(f"{LIB_PATH} has RL ABI {got}, this package needs {RL_ABI_VERSION}: rebuild it "
                               "with `python -m isaacgymenv_amd.build`")
        vp = C.c_void_p
        L.rl_gae.restype = C.c_int
        L.rl_gae.argtypes = [vp, vp, vp, vp, vp, C.c_int32, C.c_int32, C.c_double, C.c_double, vp, vp, vp, vp]
        L.rl_splitk_accum.restype = C.c_int
        L.rl_splitk_accum.argtypes = [vp, C.c_int32, C.c_int64, C.c_int32, vp, vp]
        L.rl_colsum_accum.restype = C.c_int
        L.rl_colsum_accum.argtypes = [vp, C.c_int32, C.c_int32, C.c_int32, vp, vp, vp]
        L.rl_ppo_loss.restype = C.c_int
        L.rl_ppo_loss.argtypes = [vp, C.c_int32, vp, C.c_int32, vp, vp, vp, vp, vp, vp, C.c_int32, C.c_int32,
                                  C.c_double, C.c_int32, C.c_double, C.c_double, C.c_double, vp, vp, vp, vp, vp, vp,
                                  vp]
        L.rl_ppo_loss_backward.restype = C.c_int
        L.rl_ppo_loss_backward.argtypes = [vp, vp, vp, vp, C.c_int32, C.c_int32, vp, C.c_int32, vp, C.c_int32, vp,
                                           vp]
        for f in ("rl_linear_fwd", "rl_linear_transpose", "rl_linear_bwd"):
            getattr(L, f).restype = C.c_int
        L.rl_linear_fwd.argtypes = [vp, C.c_int32, C.c_int32, C.c_int32, vp, C.c_int32, vp, C.c_int32, vp, vp]
        L.rl_linear_transpose.argtypes = [vp, C.c_int32, C.c_int32, vp, vp]
        L.rl_linear_bwd.argtypes = [vp, vp, C.c_int32, C.c_int32, vp, C.c_int32, C.c_int32, vp, vp, C.c_int32, vp, vp,
                                    C.c_int64, vp]
        for f in ("rl_linear_fwd_g", "rl_linear_bwd_g"):
            getattr(L, f).restype = C.c_int
        L.rl_linear_fwd_g.argtypes = [vp, C.c_int32, C.c_int32, C.c_int32, vp, C.c_int32, vp, C.c_int32, vp,
                                      C.POINTER(LinearGroups), vp]
        L.rl_linear_fwd_f32_g.argtypes = [vp, C.c_int32, C.c_int32, C.c_int32, vp, C.c_int32, vp, C.c_int32, vp,
                                          C.POINTER(LinearGroups), vp]
        L.rl_linear_bwd_g.argtypes = [vp, vp, C.c_int32, C.c_int32, vp, C.c_int32, C.c_int32, vp, vp, C.c_int32, vp,
                                      vp, C.c_int64, C.POINTER(LinearGroups), vp]
        L.rl_ppo_heads_partials_size.restype = C.c_int
        L.rl_ppo_heads_partials_size.argtypes = [C.c_int32, C.c_int32, C.c_int32]
        L.rl_ppo_heads_loss.restype = C.c_int
        L.rl_ppo_heads_loss.argtypes = [vp, C.c_int64, C.c_int32, C.c_int32, C.c_int32, vp, vp, vp, vp, vp, vp, vp, vp,
                                        vp, vp, C.c_int32, C.c_int32, C.c_double, C.c_int32, C.c_double, C.c_double,
                                        C.c_double, vp, vp, vp, vp, vp, vp, vp, vp]
        L.rl_ppo_heads_loss_backward.restype = C.c_int
        L.rl_ppo_heads_loss_backward.argtypes = [vp, vp, vp, vp, vp, C.c_int64, C.c_int32, C.c_int32, C.c_int32, vp, vp,
                                                 C.c_int32, C.c_int32, vp, vp, vp, vp, vp, vp, vp, C.c_int32, vp]
        L.rl_splitk_accum_multi.restype = C.c_int
        L.rl_splitk_accum_multi.argtypes = [C.POINTER(SplitkJob), C.c_int32, C.c_int32, vp]
        L.rl_policy_kl_step.restype = C.c_int
        L.rl_policy_kl_step.argtypes = [vp, C.c_int32, vp, C.c_int64, C.c_int32, vp, vp, C.c_int32, C.c_int32,
                                        C.c_int32, vp, vp, C.c_int32, C.c_double, vp, vp, vp, vp, vp, vp, vp]
        L.rl_opt_step_h.restype = C.c_int
        L.rl_opt_step_h.argtypes = [vp, vp, vp, vp, vp, C.c_int64, vp, vp, vp, vp, C.POINTER(OptHyper), vp, vp]
        L.rl_rms_normalize_h.restype = C.c_int
        L.rl_rms_normalize_h.argtypes = [vp, C.c_int32, C.c_int32, vp, vp, vp, C.c_double, C.c_int32, vp, vp, vp]
        L.rl_kl_partials_size.restype = C.c_int
        L.rl_policy_kl.restype = C.c_int
        L.rl_policy_kl.argtypes = [vp, C.c_int32, vp, C.c_int64, C.c_int32, vp, vp, C.c_int32, C.c_int32, C.c_int32, vp,
                                   vp, vp]
        L.rl_adaptive_lr.restype = C.c_int
        L.rl_adaptive_lr.argtypes = [vp, C.c_float, C.c_int32, C.c_double, vp, vp, vp, vp, vp, vp, vp]
        L.rl_opt_step.restype = C.c_int
        L.rl_opt_step.argtypes = [vp, vp, vp, vp, C.c_int64, vp, vp, vp, vp, C.POINTER(OptHyper), vp, vp]
        L.rl_opt_partials_size.restype = C.c_int
        L.rl_rms_normalize.restype = C.c_int
        L.rl_rms_normalize.argtypes = [vp, C.c_int32, C.c_int32, vp, vp, vp, C.c_double, C.c_int32, vp, vp, vp]
        L.rl_policy_head.restype = C.c_int
        L.rl_policy_head.argtypes = [vp, vp, vp, vp, vp, vp, C.c_double, C.c_int32, C.c_int32, vp, vp, vp, vp, vp]
        L.rl_rollout_post.restype = C.c_int
        L.rl_rollout_post.argtypes = [vp, vp, C.c_int32, vp, C.c_int32, vp, C.c_double, C.c_double, C.c_double,
                                      C.c_int32, vp, vp, vp, vp, vp, vp, C.c_int32, vp]
        L.rl_act_heads.restype = C.c_int
        L.rl_act_heads.argtypes = [vp, C.c_int32, vp, C.c_int32, C.c_int32, vp, vp, vp, vp, vp, vp, vp, vp, C.c_double,
                                   C.c_int32, C.c_int32, vp, vp, vp, vp, vp, vp]
        L.rl_rollout_pre.restype = C.c_int
        L.rl_rollout_pre.argtypes = [vp, C.c_int32, vp, vp, C.c_int32, vp, vp, vp, vp, C.c_int32, C.c_int32, C.c_int32,
                                     C.c_int32, vp, vp, vp, vp, vp, vp, vp, vp]
        L.rl_last_error.restype = C.c_char_p
        L.rl_abi_version.restype = C.c_int
        _lib = L
    return _lib


def _torch_discount(rewards, values, dones, last_values, last_dones, gamma, tau):
    """rl_games a2c_common.py discount_values, time-major [H, N] (CPU pipeline)."""
    H = rewards.shape[0]
    advs = torch.zeros_like(rewards)
    lastgaelam = 0
    fdones = dones.float()
    for t in reversed(range(H)):
        if t == H - 1:
            nextnonterminal = 1.0 - last_dones.float()
            nextvalues = last_values
        else:
            nextnonterminal = 1.0 - fdones[t + 1]
            nextvalues = values[t + 1]
        delta = rewards[t] + gamma * nextvalues * nextnonterminal - values[t]
        advs[t] = lastgaelam = delta + gamma * tau * nextnonterminal * lastgaelam
    return advs


def discount_values(rewards, values, dones, last_values, last_dones, gamma: float, tau: float):
    """rewards/values f32 [H, N], dones u8 [H, N], last_values f32 [N], last_dones u8 [N]
    -> (returns, advantages, values) each f32 [N * H] in env-major order (swap_and_flatten01)."""
    H, N = rewards.shape
    if rewards.device.type != "cuda":
        advs = _torch_discount(rewards, values, dones, last_values, last_dones, gamma, tau)
        returns = advs + values
        flat = lambda x: x.transpose(0, 1).reshape(-1)  # noqa: E731
        return flat(returns), flat(advs), flat(values)
    for t in (rewards, values, dones, last_values, last_dones):
        assert t.is_contiguous() and t.device == rewards.device
    assert rewards.dtype == values.dtype == last_values.dtype == torch.float32
    assert dones.dtype == last_dones.dtype == torch.uint8
    assert values.shape == dones.shape == (H, N) and last_values.shape == (N,) and last_dones.shape == (N,)
    returns = torch.empty(N * H, dtype=torch.float32, device=rewards.device)
    advs = torch.empty_like(returns)
    vals = torch.empty_like(returns)
    stream = raw_stream(rewards.device)
    rc = lib().rl_gae(rewards.data_ptr(), values.data_ptr(), dones.data_ptr(), last_values.data_ptr(),
                      last_dones.data_ptr(), H, N, float(gamma), float(tau), returns.data_ptr(), advs.data_ptr(),
                      vals.data_ptr(), stream)
    if rc != 0:
        raise RuntimeError(f"rl_gae failed: {lib().rl_last_error().decode()}")
    return returns, advs, vals


def splitk_accum(parts: torch.Tensor, grad: torch.Tensor) -> None:
    """grad += parts.sum(0) in fp32, partials added in ascending order (include/gymrl.h rl_splitk_accum).
    parts [P, ...] fp16 / f32 contiguous, grad f32 contiguous with parts[0]'s element count, both on one
    device; ordered on torch's current stream (graph-capturable)."""
    assert parts.is_cuda and grad.is_cuda and parts.device == grad.device
    assert parts.is_contiguous() and grad.is_contiguous() and grad.dtype == torch.float32
    assert parts.dtype in (torch.float16, torch.float32) and parts[0].numel() == grad.numel()
    stream = raw_stream(grad.device)
    rc = lib().rl_splitk_accum(parts.data_ptr(), parts.shape[0], grad.numel(), int(parts.dtype == torch.float16),
                               grad.data_ptr(), stream)
    if rc != 0:
        raise RuntimeError(f"rl_splitk_accum failed: {lib().rl_last_error().decode()}")


_COLSUM_WORK = {}  # device -> f32 scratch [256 * 2048], allocated before any graph capture


def colsum_supported(g: torch.Tensor) -> bool:
    return (g.is_cuda and g.dim() == 2 and g.is_contiguous() and g.dtype in (torch.float16, torch.float32)
            and g.shape[1] % 8 == 0 and g.shape[1] <= 2048 and g.data_ptr() % 16 == 0 and g.shape[0] > 0)


def colsum_accum(g: torch.Tensor, grad: torch.Tensor) -> None:
    """grad += g.sum(0) in fp32, deterministic (include/gymrl.h rl_colsum_accum); g [rows, cols] with
    colsum_supported(g), grad f32 [cols] contiguous on the same device."""
    assert colsum_supported(g) and grad.is_cuda and grad.device == g.device and grad.is_contiguous()
    assert grad.dtype == torch.float32 and grad.numel() == g.shape[1]
    ws = _COLSUM_WORK.get(g.device)
    if ws is None:
        ws = _COLSUM_WORK[g.device] = torch.empty(256 * 2048, dtype=torch.float32, device=g.device)
    stream = raw_stream(g.device)
    rc = lib().rl_colsum_accum(g.data_ptr(), g.shape[0], g.shape[1], int(g.dtype == torch.float16), grad.data_ptr(),
                               ws.data_ptr(), stream)
    if rc != 0:
        raise RuntimeError(f"rl_colsum_accum failed: {lib().rl_last_error().decode()}")


_FLAG_BYTES = {torch.bool: 1, torch.uint8: 1, torch.int64: 8}


def rollout_pre(n: int, obs, dones, values, actions, neglogp, mu, sigma, b_obs, t_dones, t_values, b_actions,
                b_neglogp, b_mu, b_sigma) -> None:
    """play_steps' experience of horizon slot n before env.step as one kernel (include/gymrl.h
    rl_rollout_pre): b_obs[:, n] = obs, t_dones[n] = dones, t_values[n] = values[:, 0], b_actions /
    b_neglogp / b_mu / b_sigma[:, n] = actions / neglogp / mu / sigma.  The caller checks layouts
    once (rollout_pre_applies); this is the per-step call."""
    N, O = obs.shape
    H, A = b_obs.shape[1], actions.shape[1]
    stream = raw_stream(obs.device)
    rc = lib().rl_rollout_pre(obs.data_ptr(), O, dones.data_ptr(), values.data_ptr(), values.stride(0),
                              actions.data_ptr(), neglogp.data_ptr(), mu.data_ptr(), sigma.data_ptr(), N, A, H, int(n),
                              b_obs.data_ptr(), t_dones.data_ptr(), t_values.data_ptr(), b_actions.data_ptr(),
                              b_neglogp.data_ptr(), b_mu.data_ptr(), b_sigma.data_ptr(), stream)
    if rc != 0:
        raise RuntimeError(lib().rl_last_error().decode())


def rollout_pre_applies(obs, dones, values, actions, neglogp, mu, sigma, b_obs, t_dones, t_values, b_actions, b_neglogp,
                        b_mu, b_sigma) -> bool:
    """The layouts rl_rollout_pre assumes (all on one GPU; the experience buffers as A2CAgent allocates them)."""
    ts = (obs, dones, values, actions, neglogp, mu, sigma, b_obs, t_dones, t_values, b_actions, b_neglogp, b_mu, b_sigma)
    if not all(isinstance(t, torch.Tensor) and t.is_cuda and t.device == obs.device for t in ts):
        return False
    N, A = actions.shape if actions.dim() == 2 else (-1, -1)
    f32 = torch.float32
    return (obs.dim() == 2 and obs.is_contiguous() and obs.dtype == f32 and dones.dtype == torch.uint8
            and dones.is_contiguous() and dones.numel() == N and values.dtype == f32 and values.dim() == 2
            and values.shape[0] == N and values.stride(1) == 1 and 0 < A <= 64
            and all(t.dtype == f32 and t.is_contiguous() and t.shape == (N, A) for t in (actions, mu, sigma))
            and neglogp.dtype == f32 and neglogp.is_contiguous() and neglogp.numel() == N
            and all(t.is_contiguous() for t in (b_obs, t_dones, t_values, b_actions, b_neglogp, b_mu, b_sigma))
            and b_obs.shape[0] == N and b_obs.shape[2] == obs.shape[1] and t_dones.dtype == torch.uint8
            and b_actions.shape == b_mu.shape == b_sigma.shape == (N, b_obs.shape[1], A))


def rollout_post(rewards, dones, time_outs, values, reward_shift: float, reward_scale: float, gamma: float,
                 dones_out, rewards_out, current_rewards, current_lengths, meter_rewards, meter_lengths,
                 games_to_track: int, outputs_checked: bool = False) -> None:
    """rl_games play_steps after env.step as one kernel (include/gymrl.h rl_rollout_post).
    rewards f32 [N]; dones / time_outs bool, uint8 or int64 [N] (time_outs None: no value bootstrap);
    values f32 [N] or [N, 1] or None; dones_out u8 [N]; rewards_out, current_* f32 [N];
    meter_* f32 [2] = (mean, current_size).  outputs_checked: the caller's own buffers (dones_out ..
    meter_lengths) passed these checks before and are unchanged -- only the env's tensors are checked
    (the per-step call of the rollout loop)."""
    N = rewards.shape[0]
    dev = rewards.device
    if dones.dtype not in _FLAG_BYTES:
        dones = dones.to(torch.uint8)
    if time_outs is not None and time_outs.dtype not in _FLAG_BYTES:
        time_outs = time_outs.to(torch.uint8)
    ins = (rewards, dones, time_outs, values)
    for t in ins if outputs_checked else ins + (dones_out, rewards_out, current_rewards, current_lengths,
                                                 meter_rewards, meter_lengths):
        if t is not None:
            assert t.is_cuda and t.device == dev and t.is_contiguous()
    assert rewards.dtype == torch.float32 and dones.numel() == N
    if not outputs_checked:
        assert rewards_out.dtype == current_rewards.dtype == current_lengths.dtype == torch.float32
        assert dones_out.dtype == torch.uint8 and dones_out.numel() == N
        assert rewards_out.numel() == N and current_rewards.numel() == N and current_lengths.numel() == N
        assert meter_rewards.numel() == 2 and meter_lengths.numel() == 2
    assert (time_outs is None) == (values is None), "value bootstrap needs both time_outs and values"
    if values is not None:
        assert values.dtype == torch.float32 and values.numel() == N and time_outs.numel() == N
    stream = raw_stream(dev)
    ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
    rc = lib().rl_rollout_post(rewards.data_ptr(), dones.data_ptr(), _FLAG_BYTES[dones.dtype], ptr(time_outs),
                               _FLAG_BYTES[time_outs.dtype] if time_outs is not None else 0, ptr(values),
                               float(reward_shift), float(reward_scale), float(gamma), N, dones_out.data_ptr(),
                               rewards_out.data_ptr(), current_rewards.data_ptr(), current_lengths.data_ptr(),
                               meter_rewards.data_ptr(), meter_lengths.data_ptr(), int(games_to_track), stream)
    if rc != 0:
        raise RuntimeError(f"rl_rollout_post failed: {lib().rl_last_error().decode()}")


class PpoLossFn(torch.autograd.Function):
    """The PPO minibatch loss (rl_ppo_loss): forward computes the loss, its four terms' means and the
    unscaled gradients in one pass; backward scales them by the upstream gradient (rl_ppo_loss_backward).
    Inputs: mu [B, A] and values [B, 1] (fp16 under autocast, or f32), logstd [A] (the sigma parameter),
    actions [B, A], old_neglogp [B], advantages [B], old_values [B, 1], returns [B, 1] (f32).
    Returns (loss 0-d, stats [4] = means of actor, critic, entropy, bound loss; not differentiable)."""

    @staticmethod
    def forward(ctx, mu, values, logstd, actions, old_neglogp, advantages, old_values, returns, e_clip: float,
                clip_value: bool, critic_coef: float, entropy_coef: float, bounds_loss_coef: float):
        B, A = mu.shape
        dev = mu.device
        for t in (mu, values, logstd, actions, old_neglogp, advantages, old_values, returns):
            assert t.is_cuda and t.device == dev and t.is_contiguous()
        assert mu.dtype in (torch.float16, torch.float32) and values.dtype in (torch.float16, torch.float32)
        assert values.numel() == B and old_values.numel() == B and returns.numel() == B and logstd.numel() == A
        assert old_neglogp.numel() == B and advantages.numel() == B and actions.shape == (B, A)
        f32 = torch.float32
        dmu = torch.empty(B, A, dtype=f32, device=dev)
        dv = torch.empty(B, dtype=f32, device=dev)
        part = torch.empty(((B + 127) // 128) * 36, dtype=f32, device=dev)
        loss = torch.empty((), dtype=f32, device=dev)
        stats = torch.empty(4, dtype=f32, device=dev)
        dls = torch.empty(A, dtype=f32, device=dev)
        stream = raw_stream(dev)
        rc = lib().rl_ppo_loss(mu.data_ptr(), int(mu.dtype == torch.float16), values.data_ptr(),
                               int(values.dtype == torch.float16), logstd.data_ptr(), actions.data_ptr(),
                               old_neglogp.data_ptr(), advantages.data_ptr(), old_values.data_ptr(), returns.data_ptr(),
                               B, A, float(e_clip), int(bool(clip_value)), float(critic_coef), float(entropy_coef),
                               float(bounds_loss_coef), dmu.data_ptr(), dv.data_ptr(), part.data_ptr(), loss.data_ptr(),
                               stats.data_ptr(), dls.data_ptr(), stream)
        if rc != 0:
            raise RuntimeError(f"rl_ppo_loss failed: {lib().rl_last_error().decode()}")
        ctx.save_for_backward(dmu, dv, dls)
        ctx.meta = (mu.dtype, values.dtype, tuple(values.shape))
        ctx.mark_non_differentiable(stats)
        return loss, stats

    @staticmethod
    def backward(ctx, g_loss, g_stats):
        dmu, dv, dls = ctx.saved_tensors
        mu_dt, v_dt, v_shape = ctx.meta
        B, A = dmu.shape
        dev = dmu.device
        g = (g_loss if g_loss is not None else torch.ones((), device=dev)).float().contiguous()
        dmu_out = torch.empty(B, A, dtype=mu_dt, device=dev)
        dv_out = torch.empty(v_shape, dtype=v_dt, device=dev)
        dls_out = torch.empty(A, dtype=torch.float32, device=dev)
        stream = raw_stream(dev)
        rc = lib().rl_ppo_loss_backward(g.data_ptr(), dmu.data_ptr(), dv.data_ptr(), dls.data_ptr(), B, A,
                                        dmu_out.data_ptr(), int(mu_dt == torch.float16), dv_out.data_ptr(),
                                        int(v_dt == torch.float16), dls_out.data_ptr(), stream)
        if rc != 0:
            raise RuntimeError(f"rl_ppo_loss_backward failed: {lib().rl_last_error().decode()}")
        return (dmu_out, dv_out, dls_out) + (None,) * 10


class HeadsSpec:
    """The mu / value heads of a separate actor-critic network for PpoHeadsLossFn: their fp16 parameter shadows and
    the f32 gradient views the learner's flat buffers give them (direct gradients), the sigma parameter's gradient,
    and where the actor / critic outputs sit in the grouped MLP's [rows][G*H] output."""

    def __init__(self, actor_col, critic_col, hidden, w_mu, b_mu, w_v, b_v, gw_mu, gb_mu, gw_v, gb_v, g_logstd,
                 store: bool = False):
        self.actor_col, self.critic_col, self.hidden = int(actor_col), int(critic_col), int(hidden)
        self.store = bool(store)  # gradients written (=), not added: the learner's zero-free flat buffer
        self.w_mu, self.b_mu, self.w_v, self.b_v = w_mu, b_mu, w_v, b_v
        self.gw_mu, self.gb_mu, self.gw_v, self.gb_v, self.g_logstd = gw_mu, gb_mu, gw_v, gb_v, g_logstd
        for t in (w_mu, b_mu, w_v, b_v):
            assert t.dtype == torch.float16 and t.is_contiguous()
        for t in (gw_mu, gb_mu, gw_v, gb_v, g_logstd):
            assert t.dtype == torch.float32 and t.is_contiguous()
        self.num_actions = w_mu.shape[0]
        assert w_mu.shape == (self.num_actions, self.hidden) and w_v.numel() == self.hidden and b_v.numel() == 1


class PpoHeadsLossFn(torch.autograd.Function):
    """The mu / value heads and the PPO loss in one pass (rl_ppo_heads_loss): hidden fp16 [B][ld] is the grouped
    actor / critic MLP output (network._GroupedMLPFn stacked); returns (loss 0-d, stats [4], mu fp16 [B][A]).  The
    backward (rl_ppo_heads_loss_backward) returns d hidden and adds the heads' and sigma's gradients straight into
    the learner's flat gradient views (HeadsSpec) -- six hipBLASLt GEMMs, two reductions, a concatenation and the
    loss's launches become four."""

    @staticmethod
    def forward(ctx, hidden, heads, logstd, actions, old_neglogp, advantages, old_values, returns, e_clip: float,
                clip_value: bool, critic_coef: float, entropy_coef: float, bounds_loss_coef: float):
        B, ld = hidden.shape
        A, H = heads.num_actions, heads.hidden
        dev = hidden.device
        assert hidden.dtype == torch.float16 and hidden.stride(1) == 1 and hidden.data_ptr() % 4 == 0
        for t in (logstd, actions, old_neglogp, advantages, old_values, returns):
            assert t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()
        assert actions.shape == (B, A) and logstd.numel() == A and old_neglogp.numel() == B
        assert advantages.numel() == B and old_values.numel() == B and returns.numel() == B
        f32 = torch.float32
        mu = torch.empty(B, A, dtype=torch.float16, device=dev)
        dmu = torch.empty(B, A, dtype=f32, device=dev)
        dv = torch.empty(B, dtype=f32, device=dev)
        part = torch.empty(lib().rl_ppo_heads_partials_size(B, H, A), dtype=f32, device=dev)
        loss = torch.empty((), dtype=f32, device=dev)
        stats = torch.empty(4, dtype=f32, device=dev)
        dls = torch.empty(A, dtype=f32, device=dev)
        stream = raw_stream(dev)
        _check(lib().rl_ppo_heads_loss(hidden.data_ptr(), hidden.stride(0), heads.actor_col, heads.critic_col, H,
                                       heads.w_mu.data_ptr(), heads.b_mu.data_ptr(), heads.w_v.data_ptr(),
                                       heads.b_v.data_ptr(), logstd.data_ptr(), actions.data_ptr(),
                                       old_neglogp.data_ptr(), advantages.data_ptr(), old_values.data_ptr(),
                                       returns.data_ptr(), B, A, float(e_clip), int(bool(clip_value)),
                                       float(critic_coef), float(entropy_coef), float(bounds_loss_coef), mu.data_ptr(),
                                       dmu.data_ptr(), dv.data_ptr(), part.data_ptr(), loss.data_ptr(),
                                       stats.data_ptr(), dls.data_ptr(), stream), "rl_ppo_heads_loss")
        ctx.save_for_backward(hidden, dmu, dv, dls, part)
        ctx.heads = heads
        ctx.set_materialize_grads(False)  # stats / mu take no gradient: no zero tensors for them
        ctx.mark_non_differentiable(stats, mu)
        return loss, stats, mu

    @staticmethod
    def backward(ctx, g_loss, g_stats, g_mu):
        hidden, dmu, dv, dls, part = ctx.saved_tensors
        hd = ctx.heads
        B, A = dmu.shape
        g = (g_loss if g_loss is not None else torch.ones((), device=hidden.device)).float().contiguous()
        dh = torch.empty_like(hidden)
        if hd.hidden * 2 != hidden.shape[1]:
            dh.zero_()  # columns outside the two ranges get no gradient
        _check(lib().rl_ppo_heads_loss_backward(g.data_ptr(), dmu.data_ptr(), dv.data_ptr(), dls.data_ptr(),
                                                hidden.data_ptr(), hidden.stride(0), hd.actor_col, hd.critic_col,
                                                hd.hidden, hd.w_mu.data_ptr(), hd.w_v.data_ptr(), B, A, dh.data_ptr(),
                                                part.data_ptr(), hd.gw_mu.data_ptr(), hd.gb_mu.data_ptr(),
                                                hd.gw_v.data_ptr(), hd.gb_v.data_ptr(), hd.g_logstd.data_ptr(),
                                                int(hd.store), raw_stream(hidden.device)),
               "rl_ppo_heads_loss_backward")
        return (dh,) + (None,) * 12


def rms_supported(x: torch.Tensor) -> bool:
    return x.is_cuda and x.dim() == 2 and x.dtype == torch.float32 and x.is_contiguous() and 0 < x.shape[1] <= 256 \
        and x.shape[0] > 0


def rms_normalize(x, running_mean, running_var, count, epsilon: float, update: bool,
                  out_half: bool = False) -> torch.Tensor:
    """RunningMeanStd forward (include/gymrl.h rl_rms_normalize): x f32 [N, C] (rms_supported), float64
    running_mean / running_var [C] and count 0-d updated in place when ``update``; returns y f32 [N, C]."""
    assert rms_supported(x)
    for t in (running_mean, running_var, count):
        assert t.dtype == torch.float64 and t.is_contiguous() and t.device == x.device
    N, Cc = x.shape
    y = torch.empty_like(x, dtype=torch.float16 if out_half else torch.float32)
    part = torch.empty(((N + 63) // 64) * Cc * 2, dtype=torch.float32, device=x.device) if update else None
    stream = raw_stream(x.device)
    fn = lib().rl_rms_normalize_h if out_half else lib().rl_rms_normalize
    rc = fn(x.data_ptr(), N, Cc, running_mean.data_ptr(), running_var.data_ptr(),
                                count.data_ptr(), float(epsilon), int(bool(update)),
                                part.data_ptr() if part is not None else None, y.data_ptr(), stream)
    if rc != 0:
        raise RuntimeError(f"rl_rms_normalize failed: {lib().rl_last_error().decode()}")
    return y


def policy_head(mu, noise, logstd, value, value_rms=None):
    """Act-forward head (include/gymrl.h rl_policy_head): returns (actions [N, A], sigmas [N, A],
    neglogp [N], values [N, 1]); value_rms: the value RunningMeanStd (value_size 1) or None."""
    N, A = mu.shape
    for t in (mu, noise, logstd, value):
        assert t.is_cuda and t.device == mu.device and t.dtype == torch.float32 and t.is_contiguous()
    assert noise.shape == mu.shape and logstd.numel() == A and value.numel() == N
    actions, sigmas = torch.empty_like(mu), torch.empty_like(mu)
    neglogp = torch.empty(N, dtype=torch.float32, device=mu.device)
    vout = torch.empty(N, 1, dtype=torch.float32, device=mu.device)
    vm = vv = None
    eps = 0.0
    if value_rms is not None:
        assert value_rms.running_mean.numel() == 1
        vm, vv, eps = value_rms.running_mean.data_ptr(), value_rms.running_var.data_ptr(), value_rms.epsilon
    stream = raw_stream(mu.device)
    rc = lib().rl_policy_head(mu.data_ptr(), noise.data_ptr(), logstd.data_ptr(), value.data_ptr(), vm, vv, float(eps),
                              N, A, actions.data_ptr(), sigmas.data_ptr(), neglogp.data_ptr(), vout.data_ptr(), stream)
    if rc != 0:
        raise RuntimeError(f"rl_policy_head failed: {lib().rl_last_error().decode()}")
    return actions, sigmas, neglogp, vout


def act_heads_applies(a_out, c_out, w_mu, b_mu, w_v, b_v, logstd) -> bool:
    """The layouts rl_act_heads takes: f32 rows on one GPU, unit column stride, one value output."""
    ts = (a_out, c_out, w_mu, b_mu, w_v, b_v, logstd)
    if not all(isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.float32 and t.device == a_out.device
               for t in ts):
        return False
    H = a_out.shape[1] if a_out.dim() == 2 else -1
    A = w_mu.shape[0]
    return (c_out.dim() == 2 and c_out.shape == a_out.shape and a_out.stride(1) == 1 and c_out.stride(1) == 1
            and w_mu.shape == (A, H) and w_mu.is_contiguous() and b_mu.numel() == A and w_v.numel() == H
            and w_v.is_contiguous() and b_v.numel() == 1 and logstd.numel() == A and logstd.is_contiguous()
            and 4 * (16 * (2 * H + 1) + (A + 1) * (H + 1) + 16 * (A + 1)) <= 64 * 1024)


def act_heads(a_out, c_out, w_mu, b_mu, w_v, b_v, noise, logstd, value_rms=None):
    """Act-forward heads + head (include/gymrl.h rl_act_heads): returns (mu [N, A], actions [N, A], sigmas [N, A],
    neglogp [N], values [N, 1]); the caller checked act_heads_applies.  noise [N, A] = torch's normal_ draws."""
    N, H = a_out.shape
    A = w_mu.shape[0]
    dev = a_out.device
    mu, actions, sigmas = (torch.empty(N, A, dtype=torch.float32, device=dev) for _ in range(3))
    neglogp = torch.empty(N, dtype=torch.float32, device=dev)
    vout = torch.empty(N, 1, dtype=torch.float32, device=dev)
    vm = vv = None
    eps = 0.0
    if value_rms is not None:
        assert value_rms.running_mean.numel() == 1
        vm, vv, eps = value_rms.running_mean.data_ptr(), value_rms.running_var.data_ptr(), value_rms.epsilon
    rc = lib().rl_act_heads(a_out.data_ptr(), a_out.stride(0), c_out.data_ptr(), c_out.stride(0), H, w_mu.data_ptr(),
                            b_mu.data_ptr(), w_v.data_ptr(), b_v.data_ptr(), noise.data_ptr(), logstd.data_ptr(), vm, vv,
                            float(eps), N, A, mu.data_ptr(), actions.data_ptr(), sigmas.data_ptr(), neglogp.data_ptr(),
                            vout.data_ptr(), raw_stream(dev))
    if rc != 0:
        raise RuntimeError(f"rl_act_heads failed: {lib().rl_last_error().decode()}")
    return mu, actions, sigmas, neglogp, vout


def opt_step(param, grad, exp_avg, exp_avg_sq, step, lr, scale, growth_tracker, hyper: OptHyper, partials) -> None:
    """The minibatch optimizer step on flat f32 buffers (include/gymrl.h rl_opt_step): unscale, found-inf,
    norm clip, Adam, GradScaler update; scale / growth_tracker None = no loss scaling."""
    rc = lib().rl_opt_step(param.data_ptr(), grad.data_ptr(), exp_avg.data_ptr(), exp_avg_sq.data_ptr(),
                           param.numel(), step.data_ptr(), lr.data_ptr(),
                           scale.data_ptr() if scale is not None else None,
                           growth_tracker.data_ptr() if growth_tracker is not None else None, C.byref(hyper),
                           partials.data_ptr(), raw_stream())
    if rc != 0:
        raise RuntimeError(f"rl_opt_step failed: {lib().rl_last_error().decode()}")


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed: {lib().rl_last_error().decode()}")


def linear_fwd(x, w_half, b_half, act: bool, out):
    """rl_linear_fwd: out [M, N] fp16 = act(x [M, K] fp16 . w_half[N, K]^T + b_half) on the matrix cores."""
    M, K = x.shape
    N = w_half.shape[0]
    _check(lib().rl_linear_fwd(x.data_ptr(), M, K, x.stride(0), w_half.data_ptr(), N,
                               b_half.data_ptr() if b_half is not None else None, int(act), out.data_ptr(),
                               raw_stream()), "rl_linear_fwd")


def linear_transpose(w_half, out):
    N, K = w_half.shape
    _check(lib().rl_linear_transpose(w_half.data_ptr(), N, K, out.data_ptr(), raw_stream()),
           "rl_linear_transpose")


def linear_bwd(dy, y, x, w, dx, splits: int, wpart, bpart, pstride: int = 0):
    """rl_linear_bwd: dx = (dy * elu'(y)) . w (w [N, K] fp16, dx None: skipped); wpart [splits, N, K] / bpart [splits, N]
    f32 row-block partials of the weight / bias gradients (finish with splitk_accum); pstride != 0: both are
    tensors / views whose blocks lie pstride floats apart (the merged [splits, N*K + N] layout)."""
    M, N = dy.shape
    K = x.shape[1]
    _check(lib().rl_linear_bwd(dy.data_ptr(), y.data_ptr(), M, N, x.data_ptr(), K, x.stride(0),
                               w.data_ptr() if w is not None else None, dx.data_ptr() if dx is not None else None,
                               splits, wpart.data_ptr() if wpart is not None else None,
                               bpart.data_ptr() if bpart is not None else None, int(pstride),
                               raw_stream()), "rl_linear_bwd")


def linear_fwd_grouped(x, ldx: int, K: int, w_half, N: int, b_half, act: bool, y, ldy: int, groups: int, x_gstride: int,
                       w_gstride: int, b_gstride: int, y_gstride: int, M: int):
    """rl_linear_fwd_g: `groups` equal-shaped layers in one launch.  Tensors are base pointers (group 0); group g's
    operands lie the given element strides further (include/gymrl.h rl_linear_groups)."""
    g = LinearGroups(groups, ldy, 0, 0, x_gstride, w_gstride, b_gstride, y_gstride, 0, 0, 0)
    _check(lib().rl_linear_fwd_g(x.data_ptr(), M, K, ldx, w_half.data_ptr(), N,
                                 b_half.data_ptr() if b_half is not None else None, int(act), y.data_ptr(), C.byref(g),
                                 raw_stream()), "rl_linear_fwd_g")


def linear_fwd_f32(x, ldx: int, K: int, w, N: int, b, act: bool, y, ldy: int, M: int, groups: int = 1,
                   x_gstride: int = 0, w_gstride: int = 0, b_gstride: int = 0, y_gstride: int = 0):
    """rl_linear_fwd_f32_g: y = act(x w^T + b) in f32 on the matrix cores, `groups` equal-shaped layers in one launch
    (tensors are base pointers of group 0; strides in elements, include/gymrl.h)."""
    g = LinearGroups(groups, ldy, 0, 0, x_gstride, w_gstride, b_gstride, y_gstride, 0, 0, 0)
    _check(lib().rl_linear_fwd_f32_g(x.data_ptr(), M, K, ldx, w.data_ptr(), N, b.data_ptr() if b is not None else None,
                                     int(act), y.data_ptr(), C.byref(g), raw_stream()),
           "rl_linear_fwd_f32_g")


def linear_bwd_grouped(dy, y, ldy: int, y_gstride: int, M: int, N: int, x, ldx: int, x_gstride: int, K: int, w,
                       w_gstride: int, dx, lddx: int, dx_gstride: int, splits: int, wpart, bpart, pstride: int,
                       part_gstride: int, bpart_gstride: int, groups: int):
    """rl_linear_bwd_g: the backward of `groups` equal-shaped layers in one launch per GEMM (dX, dW + db)."""
    g = LinearGroups(groups, ldy, lddx, 0, x_gstride, w_gstride, 0, y_gstride, dx_gstride, part_gstride, bpart_gstride)
    _check(lib().rl_linear_bwd_g(dy.data_ptr(), y.data_ptr(), M, N, x.data_ptr(), K, ldx,
                                 w.data_ptr() if w is not None else None, dx.data_ptr() if dx is not None else None,
                                 splits, wpart.data_ptr() if wpart is not None else None,
                                 bpart.data_ptr() if bpart is not None else None, int(pstride), C.byref(g),
                                 raw_stream()), "rl_linear_bwd_g")


def policy_kl(mu_new, sigma_row, mu_old, sigma_old, kl_out, partials, write_back: bool = True,
              sigma_is_log: bool = False, lr_step=None) -> None:
    """rl_policy_kl: kl_out (f32 0-d) = policy_kl(mu_new, sigma, mu_old, sigma_old) (rl_games torch_ext.policy_kl),
    sigma_new one [A] row for all rows (fixed sigma) or [M, A]; sigma_is_log: the row holds log sigma (the sigma
    parameter); write_back: mu_old / sigma_old (the dataset's rows) receive the new values
    (dataset.update_mu_sigma).  lr_step = (adaptive, kl_threshold, lr, opt_lr, stats, a_loss, c_loss, entropy):
    the single-rank minibatch's scheduler step and meters in the same launch (rl_policy_kl_step)."""
    M, A = mu_new.shape
    assert mu_new.is_contiguous() and mu_old.is_contiguous() and sigma_old.is_contiguous()
    assert mu_old.dtype == torch.float32 and sigma_old.dtype == torch.float32 and sigma_row.dtype == torch.float32
    stride = 0 if sigma_row.dim() == 1 else sigma_row.stride(0)
    stream = raw_stream()
    half = int(mu_new.dtype == torch.float16)
    if lr_step is None:
        _check(lib().rl_policy_kl(mu_new.data_ptr(), half, sigma_row.data_ptr(), stride, int(sigma_is_log),
                                  mu_old.data_ptr(), sigma_old.data_ptr(), M, A, int(write_back), kl_out.data_ptr(),
                                  partials.data_ptr(), stream), "rl_policy_kl")
        return
    adaptive, thr, lr, opt_lr, stats, a_loss, c_loss, entropy = lr_step
    ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
    _check(lib().rl_policy_kl_step(mu_new.data_ptr(), half, sigma_row.data_ptr(), stride, int(sigma_is_log),
                                   mu_old.data_ptr(), sigma_old.data_ptr(), M, A, int(write_back), kl_out.data_ptr(),
                                   partials.data_ptr(), int(adaptive), float(thr), ptr(lr), ptr(opt_lr), ptr(stats),
                                   ptr(a_loss), ptr(c_loss), ptr(entropy), stream), "rl_policy_kl_step")


def adaptive_lr(kl, inv_world: float, adaptive: bool, kl_threshold: float, lr, opt_lr, stats, a_loss, c_loss,
                entropy) -> None:
    """rl_adaptive_lr: the rank-averaged kl, AdaptiveScheduler on the f64 lr (and its f32 optimizer copy), the
    epoch meters stats[0..3] += a_loss, c_loss, kl, entropy."""
    ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
    _check(lib().rl_adaptive_lr(kl.data_ptr(), float(inv_world), int(adaptive), float(kl_threshold), ptr(lr),
                                ptr(opt_lr), ptr(stats), ptr(a_loss), ptr(c_loss), ptr(entropy),
                                raw_stream()), "rl_adaptive_lr")


def splitk_accum_multi(jobs, store: bool = False) -> None:
    """rl_splitk_accum_multi: [(parts [P, ...] f32 / fp16, grad f32)] finished in one launch (grad = / += sum)."""
    assert 0 < len(jobs) <= SPLITK_MAX_JOBS
    arr = (SplitkJob * len(jobs))()
    for k, (parts, grad) in enumerate(jobs):
        assert parts.is_contiguous() and grad.is_contiguous() and grad.dtype == torch.float32
        assert parts.dtype in (torch.float16, torch.float32) and parts[0].numel() == grad.numel()
        arr[k] = SplitkJob(parts.data_ptr(), grad.data_ptr(), grad.numel(), parts.shape[0],
                           int(parts.dtype == torch.float16))
    _check(lib().rl_splitk_accum_multi(arr, len(jobs), int(store), raw_stream()),
           "rl_splitk_accum_multi")


def opt_step_h(param, param_half, grad, exp_avg, exp_avg_sq, step, lr, scale, growth_tracker, hyper: OptHyper,
               partials) -> None:
    """rl_opt_step_h: opt_step that also writes the fp16 parameter shadow (two launches); partials zero-initialised."""
    assert param_half.dtype == torch.float16 and param_half.numel() == param.numel()
    _check(lib().rl_opt_step_h(param.data_ptr(), param_half.data_ptr(), grad.data_ptr(), exp_avg.data_ptr(),
                               exp_avg_sq.data_ptr(), param.numel(), step.data_ptr(), lr.data_ptr(),
                               scale.data_ptr() if scale is not None else None,
                               growth_tracker.data_ptr() if growth_tracker is not None else None, C.byref(hyper),
                               partials.data_ptr(), raw_stream()), "rl_opt_step_h")
