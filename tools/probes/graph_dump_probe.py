"""Dump the HIP graph of the drifting MLP forward+backward (flat-view grads, ELU, batch 8192)."""
import sys
import torch
import torch.nn as nn

dev = "cuda"
torch.manual_seed(1)
m = nn.Sequential(nn.Linear(4, 32), nn.ELU(), nn.Linear(32, 32), nn.ELU(), nn.Linear(32, 1)).to(dev)
ps = list(m.parameters())
x = torch.randn(8192, 4, device=dev)
t = torch.randn(8192, 1, device=dev)
flat = torch.zeros(sum(p.numel() for p in ps), device=dev)
off = 0
for p in ps:
    p.grad = flat[off:off + p.numel()].view_as(p)
    off += p.numel()


def fb():
    flat.zero_()
    loss = ((m(x) - t) ** 2).mean()
    loss.backward()


fb()
torch.cuda.synchronize()
ref = flat.clone()
g = torch.cuda.CUDAGraph()
g.enable_debug_mode()
with torch.cuda.graph(g):
    fb()
g.debug_dump(sys.argv[1])
for k in range(4):
    g.replay()
    torch.cuda.synchronize()
    print("replay", k, (flat - ref).abs().max().item(), flush=True)
