"""Probe: where the fused trimesh tail and the torch tail differ (obs columns / envs / reset history)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import isaacgymenv_amd  # noqa: E402,F401
from tests import test_task_gpu as T  # noqa: E402


class MP:
    def setattr(self, obj, name, val):
        setattr(obj, name, val)


env = T._make("AnymalTerrain", 256, MP(), **{"task.env.learn.episodeLength_s": 0.1, **T.TRIMESH})
gen = torch.Generator(device="cuda:0").manual_seed(9)
acts = [2 * torch.rand((256, 12), device="cuda:0", generator=gen) - 1 for _ in range(4)]
env.step(acts[0])
snap = T._snapshot(env)
kernels = env._kernels
out = {}
for mode in ("kernels", "torch"):
    T._restore(env, snap)
    env._kernels = kernels if mode == "kernels" else None
    res = []
    for a in acts:
        obs, rew, reset, extras = env.step(a)
        res.append((obs["obs"].clone(), reset.clone(), env.root_states.clone(), env.terrain_levels.clone(),
                    env.env_origins.clone(), env.measured_heights.clone(), env.commands.clone()))
    out[mode] = res
for t in range(len(acts)):
    a, b = out["kernels"][t], out["torch"][t]
    d = (a[0] - b[0]).abs()
    bad = (d > 1e-4)
    envs = bad.any(dim=1).nonzero().flatten().tolist()
    cols = bad.any(dim=0).nonzero().flatten().tolist()
    print(f"step {t}: resets {int(a[1].sum())}/{int(b[1].sum())} bad envs {envs[:20]} bad cols {cols[:40]} max {float(d.max()):.3g}")
    print("  root diff", float((a[2] - b[2]).abs().max()), "levels eq", bool(torch.equal(a[3], b[3])),
          "origins diff", float((a[4] - b[4]).abs().max()), "heights diff", float((a[5] - b[5]).abs().max()),
          "cmd diff", float((a[6] - b[6]).abs().max()))
    if envs:
        e = envs[0]
        print("  env", e, "root k", a[2][e].tolist(), "\n  root t", b[2][e].tolist())
        print("  cmd k", a[6][e].tolist(), "cmd t", b[6][e].tolist())
