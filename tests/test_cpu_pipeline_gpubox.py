"""BASELINE config 1 on the GPU box with the GPU hidden: Cartpole num_envs=64 sim_device=cpu pipeline=cpu.

The run happens in a child process whose HIP / ROCr / CUDA visible-device lists are empty, so the
product's CPU pipeline (libgymsim's host backend, gs_host.hip) is what steps it; the child checks
that no device is visible, that the sim is the host backend, and that 600 env steps (past the
500-step timeout) produce finite observations, int64 resets and bool timeouts.
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, torch
sys.path.insert(0, sys.argv[1])
import isaacgymenvs
assert torch.cuda.device_count() == 0, torch.cuda.device_count()
env = isaacgymenvs.make(seed=42, task="Cartpole", num_envs=64, sim_device="cpu", rl_device="cpu", headless=True,
                        overrides=["pipeline=cpu"])
assert env.sim.host and env.sim.kernel_variant == 3 and env.device == "cpu"
gen = torch.Generator().manual_seed(0)
resets = 0
for t in range(600):
    obs, rew, reset, extras = env.step(2 * torch.rand((64, 1), generator=gen) - 1)
    assert torch.isfinite(obs["obs"]).all() and obs["obs"].abs().max() <= 5.0
    assert reset.dtype == torch.int64 and extras["time_outs"].dtype == torch.bool
    resets += int(reset.sum())
assert resets > 0
print("cpu pipeline ok", resets)
"""


def test_cartpole64_cpu_pipeline_with_the_gpu_hidden():
    env = dict(os.environ, HIP_VISIBLE_DEVICES="", ROCR_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "cpu pipeline ok" in r.stdout
