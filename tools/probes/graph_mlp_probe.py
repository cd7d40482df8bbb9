"""Minimal MLP forward+backward under HIP-graph capture: which configuration drifts on replay?"""
import torch
import torch.nn as nn

torch.manual_seed(0)
dev = "cuda"


def make(hidden_bias=True, act=nn.ELU):
    torch.manual_seed(1)
    return nn.Sequential(nn.Linear(4, 32, bias=hidden_bias), act(), nn.Linear(32, 32, bias=hidden_bias), act(),
                         nn.Linear(32, 1)).to(dev)


def run(tag, flat_views, act=nn.ELU, loss_kind="mse", B=8192):
    m = make(act=act)
    ps = list(m.parameters())
    x = torch.randn(B, 4, device=dev)
    t = torch.randn(B, 1, device=dev)
    flat = torch.zeros(sum(p.numel() for p in ps), device=dev)
    if flat_views:
        off = 0
        for p in ps:
            p.grad = flat[off:off + p.numel()].view_as(p)
            off += p.numel()

    def fb():
        if flat_views:
            flat.zero_()
        else:
            for p in ps:
                if p.grad is not None:
                    p.grad.zero_()
        y = m(x)
        loss = ((y - t) ** 2).mean() if loss_kind == "mse" else torch.max(y - t, 0.5 * (y - t)).mean()
        loss.backward()

    def grads():
        return torch.cat([p.grad.reshape(-1) for p in ps]).clone()

    fb()
    torch.cuda.synchronize()
    ref = grads()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fb()
    out = []
    for _ in range(4):
        g.replay()
        torch.cuda.synchronize()
        d = grads() - ref
        out.append(d.abs().max().item())
    # which params drift on the last replay
    off, bad = 0, []
    for i, p in enumerate(ps):
        k = p.numel()
        if d[off:off + k].abs().max().item() > 1e-6:
            bad.append(i)
        off += k
    print(f"{tag:36s} " + " ".join(f"{v:.3g}" for v in out) + f"  drifting params {bad}", flush=True)


run("flat views, ELU", True)
run("plain grads, ELU", False)
run("flat views, ReLU", True, act=nn.ReLU)
run("flat views, Identity", True, act=nn.Identity)
run("flat views, Tanh", True, act=nn.Tanh)
run("plain grads, ReLU", False, act=nn.ReLU)
run("flat views, ELU, B=512", True, B=512)
