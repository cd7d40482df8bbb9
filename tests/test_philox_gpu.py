"""torch.rand's device stream evaluated in-kernel (csrc/torch_philox.h) is torch.rand, bit for bit.

The fused tail draws the reference's reset offsets/commands and observation noise inside its
kernels instead of launching torch's generator; these tests pin that stream and the generator
bookkeeping (offset increments) against torch itself on the GPU, for sizes that take one and
several grid-stride iterations, and the full AnymalTerrain tail in both draw modes.
"""
import ctypes as C

import pytest
import torch

pytestmark = pytest.mark.gpu

SIZES = [1, 3, 12, 255, 256, 257, 4096, 4096 * 12, 4096 * 188, 2048 * 256 * 4 + 7, 5_000_003]


@pytest.mark.parametrize("n", SIZES)
def test_inkernel_stream_equals_torch_rand(n):
    from isaacgymenv_amd import gymtask
    L = gymtask.lib()
    planner = gymtask.TorchRandPlanner("cuda:0")
    g = planner.gen
    g.manual_seed(1234 + n)
    torch.rand(1001, device="cuda:0")  # move the offset off zero
    off0 = g.get_offset()
    plan = planner.plan(n)
    off1 = g.get_offset()
    out = torch.empty(n, device="cuda:0")
    assert L.gt_torch_rand(C.byref(plan), C.c_void_p(out.data_ptr()), None) == 0
    g.set_offset(off0)
    ref = torch.rand(n, device="cuda:0")
    assert g.get_offset() == off1, "generator offset must advance exactly as torch's"
    torch.cuda.synchronize()
    assert torch.equal(out, ref)


def test_tail_inkernel_draws_equal_torch_drawn_buffers(monkeypatch):
    """Same env state, same generator position: the kernel tail with in-kernel draws and with
    torch-drawn buffers agree bit for bit, over steps with resets."""
    from tests.test_task_gpu import _make, _restore, _snapshot
    n = 256
    env = _make("AnymalTerrain", n, monkeypatch, **{"task.env.learn.episodeLength_s": 0.1})
    gen = torch.Generator(device="cuda:0").manual_seed(4)
    acts = [2 * torch.rand((n, 12), device="cuda:0", generator=gen) - 1 for _ in range(10)]
    env.step(acts[0])
    snap = _snapshot(env)
    out = {}
    for inkernel in (True, False):
        _restore(env, snap)
        env._kernels.inkernel_rng = inkernel
        res = []
        for a in acts:
            obs, rew, reset, extras = env.step(a)
            res.append((obs["obs"].clone(), rew.clone(), reset.clone(), env.root_states.clone(),
                        env.dof_state.clone(), env.commands.clone()))
        out[inkernel] = (res, torch.cuda.default_generators[0].get_offset())
    env._kernels.inkernel_rng = True
    assert out[True][1] == out[False][1]
    resets = 0
    for t, (a, b) in enumerate(zip(out[True][0], out[False][0])):
        resets += int(bool(a[2].any()))
        for x, y, what in zip(a, b, ("obs", "rew", "reset", "root", "dof", "commands")):
            assert torch.equal(x, y), f"{what} step {t}"
    assert resets >= 2
