"""Host-side (Python) cost of VecTask.step on the GPU pipeline, by function (cProfile).

    python tools/host_profile.py [--steps 300] [--num-envs 4096]
"""
import argparse
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--num-envs", type=int, default=4096)
    ap.add_argument("--episode-s", type=float, default=None, help="short episodes: every step resets")
    a = ap.parse_args()
    import torch
    import isaacgymenvs
    ov = [] if a.episode_s is None else [f"task.env.learn.episodeLength_s={a.episode_s}"]
    env = isaacgymenvs.make(seed=42, task="AnymalTerrain", num_envs=a.num_envs, sim_device="cuda:0",
                            rl_device="cuda:0", headless=True, force_render=False, overrides=ov)
    N, A = env.num_envs, env.num_actions
    pool = torch.empty((64, N, A), device="cuda:0").uniform_(-1, 1)
    for i in range(50):
        env.step(pool[i % 64])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        env.step(pool[i % 64])
    torch.cuda.synchronize()
    print(f"plain: {(time.perf_counter() - t0) / a.steps * 1e6:.1f} us/step")
    pr = cProfile.Profile()
    pr.enable()
    for i in range(a.steps):
        env.step(pool[i % 64])
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
