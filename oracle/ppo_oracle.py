"""PPO learner oracle -- TEST INFRASTRUCTURE ONLY (imported by tests/ alone).

numpy restatement of rl_games' ``A2CBase.discount_values`` (rl_games/common/a2c_common.py,
rl-games 1.6.x; the reference requires rl-games>=1.6.0 at setup.py:22 and calls it through
isaacgymenvs/train.py:188-218 -- rl_games is absent from /root/reference and from this image,
so this restatement is PARITY UNPINNED against rl_games itself: no reference test or fixture
covers the learner).  float32 throughout, same association order as the torch loop, so the
result is bit-comparable with the HIP kernel (libgymrl.so, built with -ffp-contract=off).

Also the RunningMeanStd moment merge (rl_games/algos_torch/running_mean_std.py) in float64.
"""
from __future__ import annotations

import numpy as np


def discount_values(rewards, values, dones, last_values, last_dones, gamma: float, tau: float):
    """rewards/values f32 [H,N], dones u8 [H,N], last_* [N] -> advantages f32 [H,N]."""
    H = rewards.shape[0]
    f32 = np.float32
    g = f32(gamma)
    gt = f32(gamma * tau)
    advs = np.zeros_like(rewards, dtype=f32)
    lastgaelam = np.zeros(rewards.shape[1], dtype=f32)
    for t in reversed(range(H)):
        if t == H - 1:
            nn = f32(1.0) - last_dones.astype(f32)
            nv = last_values.astype(f32)
        else:
            nn = f32(1.0) - dones[t + 1].astype(f32)
            nv = values[t + 1]
        delta = (rewards[t] + (g * nv) * nn) - values[t]
        lastgaelam = delta + (gt * nn) * lastgaelam
        advs[t] = lastgaelam
    return advs


def env_major(x):
    """swap_and_flatten01: [H, N, ...] -> [N*H, ...]."""
    return np.ascontiguousarray(np.swapaxes(x, 0, 1)).reshape((x.shape[0] * x.shape[1],) + x.shape[2:])


def rms_merge(mean, var, count, batch):
    """RunningMeanStd._update_mean_var_count_from_moments with torch.var (unbiased) batch moments."""
    batch = batch.astype(np.float64)
    bm = batch.mean(0)
    bv = batch.var(0, ddof=1)
    bc = batch.shape[0]
    delta = bm - mean
    tot = count + bc
    new_mean = mean + delta * bc / tot
    m2 = var * count + bv * bc + delta ** 2 * count * bc / tot
    return new_mean, m2 / tot, tot
