"""Probe: is the trimesh AnymalTerrain rollout bit-deterministic run to run (same seeds, same process)?
Prints the first step where two runs' root states differ, and the first non-finite root per run.

    python tools/probes/trimesh_determinism.py [steps]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def run(steps, extra_reads):
    import isaacgymenvs
    from isaacgymenv_amd.isaacgymenvs.tasks.base import vec_task
    vec_task.EXISTING_SIM = None
    dev = "cuda:0"
    env = isaacgymenvs.make(seed=42, task="AnymalTerrain", num_envs=4096, sim_device=dev, rl_device=dev,
                            graphics_device_id=-1, headless=True, force_render=False,
                            overrides=["task.env.terrain.terrainType=trimesh"])
    env.reset()
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    roots, first_bad = [], None
    for t in range(steps):
        a = torch.empty((env.num_envs, env.num_actions), device=dev).uniform_(-1, 1, generator=g)
        if extra_reads:
            _ = env.root_states.clone(), env.dof_state.clone()
        env.step(a)
        r = env.root_states.clone()
        roots.append(r.cpu())
        bad = ~torch.isfinite(r).all(dim=1)
        if first_bad is None and bad.any():
            first_bad = (t, torch.nonzero(bad).flatten().tolist()[:8])
    del env
    torch.cuda.empty_cache()
    return roots, first_bad


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    ra, ba = run(steps, False)
    rb, bb = run(steps, False)
    rc, bc = run(steps, True)
    print("first non-finite root: run A", ba, "run B", bb, "run C (extra reads)", bc, flush=True)
    for name, other in (("B", rb), ("C", rc)):
        for t in range(steps):
            if not torch.equal(torch.nan_to_num(ra[t], nan=1e30), torch.nan_to_num(other[t], nan=1e30)):
                d = (torch.nan_to_num(ra[t]) - torch.nan_to_num(other[t])).abs().amax(dim=1)
                envs = torch.nonzero(d > 0).flatten().tolist()
                print(f"A vs {name}: first difference at step {t}, {len(envs)} envs, e.g. {envs[:8]}, "
                      f"max {float(d.max()):.3g}", flush=True)
                break
        else:
            print(f"A vs {name}: bit-identical over {steps} steps", flush=True)


if __name__ == "__main__":
    main()
