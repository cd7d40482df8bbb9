"""Replays a captured minibatch forward+backward and compares the flat gradient with eager.

python tools/graph_grad_probe.py [zero_mode]   zero_mode: zero | mul | outside"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from isaacgymenv_amd.isaacgymenvs.config import compose  # noqa: E402
from isaacgymenv_amd.isaacgymenvs.tasks.base import vec_task  # noqa: E402
from isaacgymenv_amd.rl import A2CAgent, PpoConfig  # noqa: E402
import isaacgymenvs  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "zero"
vec_task.EXISTING_SIM = None
cfg = compose("config", ["task=Cartpole"])
env = isaacgymenvs.make(seed=42, task="Cartpole", num_envs=512, sim_device="cuda:0", rl_device="cuda:0",
                        headless=True, force_render=False)
agent = A2CAgent(env, PpoConfig.from_train_cfg(cfg["train"]), device="cuda:0", seed=42, use_graphs=False)
agent.train_epoch()
agent.train_epoch()
agent.model.train()
agent.model.running_mean_std.eval()  # frozen input stats: every call sees the same normalised batch

if mode == "mul":
    agent.flat_grad.zero_ = lambda: agent.flat_grad.mul_(0.0)  # type: ignore[method-assign]


def fb():
    if mode == "outside":
        out = agent._mb_forward_backward.__wrapped__(agent, 0) if hasattr(agent._mb_forward_backward, "__wrapped__") \
            else agent._mb_forward_backward(0)
    else:
        out = agent._mb_forward_backward(0)
    return out


fb()
torch.cuda.synchronize()
ref = agent.flat_grad.clone()
print("eager ref norm", ref.norm().item(), flush=True)
fb()
torch.cuda.synchronize()
print("eager repeat maxdiff", (agent.flat_grad - ref).abs().max().item(), flush=True)

torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, pool=torch.cuda.graph_pool_handle()):
    fb()
torch.cuda.synchronize()
for k in range(12):
    if mode == "outside":
        agent.flat_grad.zero_()
    g.replay()
    torch.cuda.synchronize()
    d = (agent.flat_grad - ref).abs().max().item()
    print(f"replay {k} norm {agent.flat_grad.norm().item():.6g} maxdiff {d:.3g}", flush=True)

names = [n for n, _ in agent.model.named_parameters()]
off = 0
for n, p in zip(names, agent.params):
    k = p.numel()
    print(f"  {n:40s} {tuple(p.shape)} maxdiff {(agent.flat_grad[off:off+k] - ref[off:off+k]).abs().max().item():.3g}")
    off += k

# forward-only graph: compare the loss pieces across replays
agent.flat_grad.zero_()
with torch.no_grad():
    eo = [t.clone() for t in agent.model({"is_train": True, "prev_actions": agent.dataset["actions"][:8192],
                                           "obs": agent.dataset["obs"][:8192]}).values()]
gf = torch.cuda.CUDAGraph()
with torch.cuda.graph(gf, pool=torch.cuda.graph_pool_handle()):
    with torch.no_grad():
        fo = list(agent.model({"is_train": True, "prev_actions": agent.dataset["actions"][:8192],
                               "obs": agent.dataset["obs"][:8192]}).values())
for k in range(3):
    gf.replay()
    torch.cuda.synchronize()
    print("fwd replay", k, [f"{(a - b).abs().max().item():.3g}" for a, b in zip(fo, eo)], flush=True)

# same with a 2-graph split: zero in one graph, backward in another
g2 = torch.cuda.CUDAGraph()
with torch.cuda.graph(g2, pool=torch.cuda.graph_pool_handle()):
    agent.flat_grad.zero_()
    agent._stats_acc.add_(1.0)
torch.cuda.synchronize()
g2.replay()
torch.cuda.synchronize()
print("zero graph leaves norm", agent.flat_grad.norm().item(), flush=True)
