"""Where a PPO rollout step's wall time goes on the host (GPU box probe).

Wraps the rollout's host-side calls with perf_counter accumulators and reports microseconds per
horizon step: the time the host spends inside each call (including the blocking wait on post_a's
reset count) and the rest of play_steps.  Usage: python tools/probes/rollout_host.py [--epochs 3]
"""
import argparse
import collections
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--num-envs", type=int, default=4096)
    ap.add_argument("--cprofile", action="store_true", help="also run 2 epochs under cProfile (top 40 by tottime)")
    args = ap.parse_args()
    import torch
    import isaacgymenvs
    from isaacgymenv_amd.isaacgymenvs.config import compose
    from isaacgymenv_amd.rl import A2CAgent, PpoConfig
    dev = "cuda:0"
    env = isaacgymenvs.make(seed=42, task="AnymalTerrain", num_envs=args.num_envs, sim_device=dev, rl_device=dev,
                            graphics_device_id=-1, headless=True, force_render=False)
    train = compose("config", ["task=AnymalTerrain"])["train"]
    agent = A2CAgent(env, PpoConfig.from_train_cfg(train, multi_gpu=False), device=dev, seed=42)
    agent.env_reset()
    agent.train_epoch()
    acc = collections.Counter()

    def wrap(obj, name, key):
        f = getattr(obj, name)

        def g(*a, **k):
            t0 = time.perf_counter()
            try:
                return f(*a, **k)
            finally:
                acc[key] += time.perf_counter() - t0
        setattr(obj, name, g)

    task = env
    wrap(agent, "get_action_values", "get_action_values")
    wrap(agent, "_store_post_fused", "store_post_fused")
    wrap(task, "step", "env.step")
    wrap(task, "fused_physics_step", "  fused_physics_step")
    wrap(task, "post_physics_step", "  post_physics_step")
    kern = task._kernels
    wrap(kern, "post_a", "    post_a")
    wrap(kern, "observe", "    observe")
    wrap(kern, "wait_reset_count", "    wait_reset_count (blocked)")
    wrap(kern, "reset_flagged", "    reset_flagged")
    wrap(kern, "rng_snapshot", "    rng_snapshot")
    from isaacgymenv_amd import gymtask
    L = gymtask.lib()
    for fn in ("gt_anymal_reset_flagged", "gt_anymal_post_physics_b", "gt_anymal_post_physics_a"):
        if hasattr(L, fn):
            wrap(L, fn, "      C " + fn)
    wrap(task, "_set_reset_state", "      _set_reset_state")
    wrap(kern.planner, "plan_many", "      plan_many")
    steps = 0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.epochs):
        agent.play_steps()
        steps += agent.horizon
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    out = {"us_per_step_wall": 1e6 * wall / steps}
    for k, v in acc.items():
        out[k] = 1e6 * v / steps
    print(json.dumps(out, indent=1))
    if args.cprofile:
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(2):
            agent.play_steps()
        torch.cuda.synchronize()
        pr.disable()
        pstats.Stats(pr, stream=sys.stdout).sort_stats("tottime").print_stats(45)


if __name__ == "__main__":
    main()
