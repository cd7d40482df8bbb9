"""rl_games ``algos_torch/running_mean_std.py`` RunningMeanStd (rl-games 1.6.x semantics).

float64 running moments, merged per forward call in train mode with the parallel-variance
formula (batch variance is torch's unbiased ``var``); normalised output clamped to [-5, 5];
``unnorm=True`` clamps the input to [-5, 5] then maps back.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import gae


class RunningMeanStd(nn.Module):
    def __init__(self, insize, epsilon: float = 1e-05, norm_only: bool = False):
        super().__init__()
        self.insize = insize
        self.epsilon = epsilon
        self.norm_only = norm_only
        self.axis = [0]
        self.register_buffer("running_mean", torch.zeros(insize, dtype=torch.float64))
        self.register_buffer("running_var", torch.ones(insize, dtype=torch.float64))
        self.register_buffer("count", torch.ones((), dtype=torch.float64))

    @staticmethod
    def _update_mean_var_count_from_moments(mean, var, count, batch_mean, batch_var, batch_count):
        delta = batch_mean - mean
        tot_count = count + batch_count
        new_mean = mean + delta * batch_count / tot_count
        m_a = var * count
        m_b = batch_var * batch_count
        m2 = m_a + m_b + delta ** 2 * count * batch_count / tot_count
        new_var = m2 / tot_count
        return new_mean, new_var, tot_count

    def forward_half(self, input):
        """forward(input) rounded to fp16 (train or eval mode as forward)."""
        if not self.norm_only and gae.rms_supported(input):
            return gae.rms_normalize(input, self.running_mean, self.running_var, self.count, self.epsilon,
                                     update=self.training, out_half=True)
        return self.forward(input).to(torch.float16)

    def forward(self, input, unnorm: bool = False):
        if not unnorm and not self.norm_only and gae.rms_supported(input):
            # device path: the moment update and the normalisation as one HIP pass (rl_rms_normalize)
            return gae.rms_normalize(input, self.running_mean, self.running_var, self.count, self.epsilon,
                                     update=self.training)
        if self.training:
            mean = input.mean(self.axis)
            var = input.var(self.axis)
            new_mean, new_var, new_count = self._update_mean_var_count_from_moments(
                self.running_mean, self.running_var, self.count, mean, var, input.size()[0])
            # in place (rl_games rebinds the buffers): the update is then replayable in a HIP graph
            self.running_mean.copy_(new_mean)
            self.running_var.copy_(new_var)
            self.count.copy_(new_count)
        current_mean, current_var = self.running_mean, self.running_var
        if unnorm:
            y = torch.clamp(input, min=-5.0, max=5.0)
            return torch.sqrt(current_var.float() + self.epsilon) * y + current_mean.float()
        if self.norm_only:
            return input / torch.sqrt(current_var.float() + self.epsilon)
        y = (input - current_mean.float()) / torch.sqrt(current_var.float() + self.epsilon)
        return torch.clamp(y, min=-5.0, max=5.0)
