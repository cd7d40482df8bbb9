"""A/B: fused capturable Adam + unscale + grad-norm clip over the actor-critic's 17 parameter tensors
vs over ONE flat tensor (the learner's layout), AnymalTerrainPPO network sizes.
    python tools/probes/flat_adam_ab.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

from isaacgymenv_amd.rl.network import ActorCriticNetwork  # noqa: E402

net = ActorCriticNetwork(188, 12, [512, 256, 128]).cuda()
params = list(net.parameters())
for p in params:
    p.grad = torch.randn_like(p) * 1e-3
flat = nn.Parameter(torch.cat([p.detach().reshape(-1) for p in params]), requires_grad=False)
flat.grad = torch.cat([p.grad.reshape(-1) for p in params])
lr = torch.tensor(3e-4, device="cuda")


def t(fn, reps=300):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return 1e6 * (time.perf_counter() - t0) / reps


out = {}
for name, ps in (("per_tensor", params), ("flat", [flat])):
    opt = torch.optim.Adam(ps, lr=lr, eps=1e-8, fused=True, capturable=True)
    scaler = torch.amp.GradScaler("cuda")
    scaler.scale(torch.ones((), device="cuda"))  # initialises the scale as a training step would

    def step():
        scaler.unscale_(opt)
        nn.utils.clip_grad_norm_(ps, 1.0)
        scaler.step(opt)
        scaler.update()
        scaler.scale(torch.ones((), device="cuda"))
    out[f"{name}_step_us"] = t(step)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    out[f"{name}_graph_us"] = t(g.replay)
print(out, flush=True)
