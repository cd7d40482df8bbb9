"""Host time from post_a's count arriving (the wait call returning) to the next physics launch's C call, per
headline bench step (GPU box probe): the part of the step the GPU idles for.  Also cProfile of the same loop.
    python tools/probes/post_wake.py [--steps 300]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    a = ap.parse_args()
    import torch
    import isaacgymenvs
    from isaacgymenv_amd.isaacgym import _lib
    env = isaacgymenvs.make(seed=42, task="AnymalTerrain", num_envs=4096, sim_device="cuda:0", rl_device="cuda:0",
                            graphics_device_id=-1, headless=True, force_render=False)
    env.reset()
    pool = torch.empty((64, env.num_envs, env.num_actions), device="cuda:0").uniform_(-1, 1)
    kern = env._kernels
    marks = {"wake": None}
    spans = []
    real_wait = kern.wait_reset_observe

    def wait(snap):
        k = real_wait(snap)
        marks["wake"] = time.perf_counter()
        return k
    kern.wait_reset_observe = wait
    L = _lib.lib()
    real_pd = L.gs_sim_pd_step

    def pd(*args):
        if marks["wake"] is not None:
            spans.append(time.perf_counter() - marks["wake"])
        return real_pd(*args)
    L.gs_sim_pd_step = pd
    for i in range(a.steps):
        env.step(pool[i % 64])
    torch.cuda.synchronize()
    spans.sort()
    n = len(spans)
    print(f"wake -> next pd_step C call: median {1e6 * spans[n // 2]:.1f} us, p10 {1e6 * spans[n // 10]:.1f}, "
          f"p90 {1e6 * spans[9 * n // 10]:.1f} ({n} steps)")
    import cProfile
    import pstats
    pr = cProfile.Profile()
    pr.enable()
    for i in range(200):
        env.step(pool[i % 64])
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr, stream=sys.stdout).sort_stats("tottime").print_stats(30)


if __name__ == "__main__":
    main()
