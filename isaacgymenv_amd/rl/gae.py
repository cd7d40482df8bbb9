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

LIB_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_lib", "libgymrl.so")
EXPORTED_SYMBOLS = ["rl_abi_version", "rl_last_error", "rl_gae"]
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build it with `python -m isaacgymenv_amd.build`. "
                               "Device tensors have no torch fallback for GAE.")
        L = C.CDLL(LIB_PATH)
        vp = C.c_void_p
        L.rl_gae.restype = C.c_int
        L.rl_gae.argtypes = [vp, vp, vp, vp, vp, C.c_int32, C.c_int32, C.c_double, C.c_double, vp, vp, vp, vp]
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
    stream = torch.cuda.current_stream(rewards.device).cuda_stream
    rc = lib().rl_gae(rewards.data_ptr(), values.data_ptr(), dones.data_ptr(), last_values.data_ptr(),
                      last_dones.data_ptr(), H, N, float(gamma), float(tau), returns.data_ptr(), advs.data_ptr(),
                      vals.data_ptr(), stream)
    if rc != 0:
        raise RuntimeError(f"rl_gae failed: {lib().rl_last_error().decode()}")
    return returns, advs, vals
