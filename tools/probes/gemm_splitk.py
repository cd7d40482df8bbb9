"""Probe: weight-gradient GEMMs of the PPO learner (reduction over the 16384-row minibatch):
one GEMM vs split-K as a batched GEMM + sum, fp16."""
import torch

dev = "cuda:0"
B = 16384


def t(fn, n=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / n * 1e3


for (n, k) in [(512, 188), (256, 512), (128, 256), (12, 128), (1, 128)]:
    g = torch.randn(B, n, device=dev, dtype=torch.float16)
    x = torch.randn(B, k, device=dev, dtype=torch.float16)
    base = t(lambda: g.t() @ x)
    ref = (g.float().t() @ x.float())
    res = [f"N={n:4d} K={k:4d} g^T x {base:7.1f} us"]
    for S in (8, 16, 32, 64):
        f = lambda: torch.bmm(g.view(S, B // S, n).transpose(1, 2), x.view(S, B // S, k)).sum(0, dtype=torch.float32)
        tt = t(f)
        err = float((f() - ref).abs().max() / ref.abs().max())
        res.append(f"S{S} {tt:6.1f} us (rel {err:.1e})")
    print("  ".join(res))
