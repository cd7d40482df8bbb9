"""Probe: time the PPO learner's GEMM shapes (AnymalTerrainPPO: minibatch 16384, MLP 188-512-256-128)
in fp16 with torch.nn.functional.linear and its backward, aligned vs unaligned feature widths."""
import torch
import torch.nn.functional as F

dev = "cuda:0"
B = 16384


def t(fn, n=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / n * 1e3


for (k, n) in [(188, 512), (192, 512), (512, 256), (256, 128), (128, 12), (128, 16), (128, 1), (128, 8)]:
    x = torch.randn(B, k, device=dev, dtype=torch.float16, requires_grad=True)
    w = torch.randn(n, k, device=dev, dtype=torch.float16, requires_grad=True)
    b = torch.randn(n, device=dev, dtype=torch.float16, requires_grad=True)
    y = F.linear(x, w, b)
    g = torch.randn_like(y)
    fwd = t(lambda: F.linear(x, w, b))
    bwd = t(lambda: torch.autograd.grad(F.linear(x, w, b), (x, w, b), g))
    fl = 2 * B * k * n
    print(f"K={k:4d} N={n:4d}  fwd {fwd:8.1f} us ({fl / fwd / 1e6:7.1f} TF/s)   fwd+bwd {bwd:8.1f} us")
