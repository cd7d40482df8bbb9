"""A/B of the learner's gradient-finish kernels vs the torch ops they replace (MI355X, one process):
bias column sums (rl_colsum_accum vs g.sum(0, fp32) + .grad add), split-K finish (rl_splitk_accum vs
parts.sum(0, fp32) + add), fp16 weight casts (one flat cast vs one cast per tensor).
    python tools/probes/grad_kernels_ab.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from isaacgymenv_amd.rl import gae  # noqa: E402


def t(fn, reps=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return 1e6 * (time.perf_counter() - t0) / reps


out = {}
for cols in (512, 256, 128):
    g = torch.randn(16384, cols, device="cuda").half()
    grad = torch.zeros(cols, device="cuda")
    out[f"bias{cols}_torch_us"] = t(lambda: grad.add_(g.sum(0, dtype=torch.float32)))
    out[f"bias{cols}_kernel_us"] = t(lambda: gae.colsum_accum(g, grad))
for n, k in ((512, 188), (256, 512), (128, 256)):
    parts = torch.randn(16, n, k, device="cuda").half()
    grad = torch.zeros(n, k, device="cuda")
    out[f"splitk{n}x{k}_torch_us"] = t(lambda: grad.add_(parts.sum(0, dtype=torch.float32)))
    out[f"splitk{n}x{k}_kernel_us"] = t(lambda: gae.splitk_accum(parts, grad))
shapes = [(512, 188), (512,), (256, 512), (256,), (128, 256), (128,)] * 2 + [(1, 128), (1,), (12, 128), (12,)]
ps = [torch.randn(s, device="cuda") for s in shapes]
flat = torch.cat([p.reshape(-1) for p in ps])
half = torch.empty_like(flat, dtype=torch.float16)
out["casts_per_tensor_us"] = t(lambda: [p.half() for p in ps])
out["cast_flat_us"] = t(lambda: half.copy_(flat))
print(out, flush=True)
