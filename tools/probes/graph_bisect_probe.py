"""Bisect the replay drift of a captured MLP forward+backward (tools/graph_mlp_probe.py)."""
import sys
import torch
import torch.nn as nn
import torch.nn.functional as F

dev = "cuda"


class BiasAfter(nn.Linear):
    def forward(self, x):
        return F.linear(x, self.weight) + self.bias


def run(tag, views=True, lin=nn.Linear, zero="flat", B=8192, blas=None):
    if blas:
        torch.backends.cuda.preferred_blas_library(blas)
    torch.manual_seed(1)
    m = nn.Sequential(lin(4, 32), nn.ELU(), lin(32, 32), nn.ELU(), lin(32, 1)).to(dev)
    ps = list(m.parameters())
    x = torch.randn(B, 4, device=dev)
    t = torch.randn(B, 1, device=dev)
    flat = torch.zeros(sum(p.numel() for p in ps), device=dev)
    grads = []
    off = 0
    for p in ps:
        p.grad = flat[off:off + p.numel()].view_as(p) if views else torch.zeros_like(p)
        grads.append(p.grad)
        off += p.numel()

    def fb():
        if zero == "flat":
            flat.zero_()
        elif zero == "foreach":
            torch._foreach_zero_(grads)
        else:
            for gr in grads:
                gr.zero_()
        loss = ((m(x) - t) ** 2).mean()
        loss.backward()

    def cat():
        return torch.cat([p.grad.reshape(-1) for p in ps]).clone()

    fb()
    torch.cuda.synchronize()
    ref = cat()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fb()
    worst, bad = 0.0, set()
    for _ in range(4):
        g.replay()
        torch.cuda.synchronize()
        d = cat() - ref
        worst = max(worst, d.abs().max().item())
        o = 0
        for i, p in enumerate(ps):
            if d[o:o + p.numel()].abs().max().item() > 1e-5:
                bad.add(i)
            o += p.numel()
    print(f"{tag:40s} worst {worst:.3g} drifting {sorted(bad)}", flush=True)
    if blas:
        torch.backends.cuda.preferred_blas_library("default")


if len(sys.argv) > 1 and sys.argv[1] == "repeat":
    for k in range(8):
        run(f"views flat-zero #{k}")
        run(f"plain foreach, bias-after #{k}", views=False, zero="foreach", lin=BiasAfter)
    sys.exit(0)
run("views flat-zero")
run("views flat-zero again")
run("views per-zero", zero="per")
run("plain per-zero", views=False, zero="per")
run("plain foreach-zero", views=False, zero="foreach")
run("views, bias-after linear", lin=BiasAfter)
run("plain foreach, bias-after", views=False, zero="foreach", lin=BiasAfter)
run("views, rocblas", blas="cublas")
run("plain foreach, rocblas", views=False, zero="foreach", blas="cublas")
run("views, hipblaslt", blas="cublaslt")
run("views B=2048", B=2048)
run("views B=4096", B=4096)
run("views B=16384", B=16384)
