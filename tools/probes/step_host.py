"""Where a bench step's wall time goes on the host (GPU box probe): AnymalTerrain 4096 envs, uniform random
actions, the bench's loop.  Wraps the host-side calls of VecTask.step with perf_counter accumulators and
reports microseconds per step (time inside each call, including the blocking wait on post_a's reset count),
the share of steps that reset envs, and optionally a cProfile of the loop.

    python tools/probes/step_host.py [--steps 500] [--cprofile]
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
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--num-envs", type=int, default=4096)
    ap.add_argument("--cprofile", action="store_true")
    args = ap.parse_args()
    import torch
    import isaacgymenvs
    dev = "cuda:0"
    env = isaacgymenvs.make(seed=42, task="AnymalTerrain", num_envs=args.num_envs, sim_device=dev, rl_device=dev,
                            graphics_device_id=-1, headless=True, force_render=False)
    N, A = env.num_envs, env.num_actions
    pool = torch.empty((64, N, A), device=dev).uniform_(-1, 1)
    for i in range(args.warmup):
        env.step(pool[i % 64])
    acc = collections.Counter()
    resets = [0, 0]

    def wrap(obj, name, key):
        f = getattr(obj, name)

        def g(*a, **k):
            t0 = time.perf_counter()
            try:
                return f(*a, **k)
            finally:
                acc[key] += time.perf_counter() - t0
        setattr(obj, name, g)

    kern = env._kernels
    wrap(env, "fused_physics_step", "  fused_physics_step")
    wrap(env, "post_physics_step", "  post_physics_step")
    wrap(kern, "post_a", "    post_a")
    wrap(kern, "observe", "    observe")
    wrap(kern, "wait_reset_count", "    wait_reset_count (blocked)")
    wrap(kern, "reset_flagged", "    reset_flagged")
    wrap(kern, "finish_reset", "    finish_reset")
    wrap(env, "_set_reset_state", "      _set_reset_state")
    wrap(kern.planner, "plan_many", "      plan_many")
    orig_wait = kern.wait_reset_count

    def counting_wait():
        k = orig_wait()
        resets[0] += k > 0
        resets[1] += k
        return k
    kern.wait_reset_count = counting_wait
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        t1 = time.perf_counter()
        env.step(pool[i % 64])
        acc["env.step"] += time.perf_counter() - t1
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    out = {"us_per_step_wall": 1e6 * wall / args.steps, "reset_steps_frac": resets[0] / args.steps,
           "envs_reset_per_step": resets[1] / args.steps}
    for k, v in sorted(acc.items()):
        out[k] = 1e6 * v / args.steps
    print(json.dumps(out, indent=1))
    if args.cprofile:
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        for i in range(200):
            env.step(pool[i % 64])
        torch.cuda.synchronize()
        pr.disable()
        pstats.Stats(pr, stream=sys.stdout).sort_stats("tottime").print_stats(40)


if __name__ == "__main__":
    main()
