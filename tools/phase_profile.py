"""Per-phase cycle breakdown of the lane-team physics kernel (profiling build).

    python -m isaacgymenv_amd.build && python tools/phase_profile.py [--steps 100]

Loads libgymsim_prof.so (-DGS_PHASE_PROFILE) instead of libgymsim.so, runs AnymalTerrain
steps and prints, per kernel launch and wave, the s_memtime cycles of each solver phase and the
number of contacts each wave executes in the PGS sweeps (wave-uniform control flow: a contact
costs a wave its full latency if ANY of its 16 envs has it active).
"""
import argparse
import ctypes as C
import os
import sys

os.environ.setdefault("GS_LIBGYMSIM", "libgymsim_prof.so")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PHASES = ["forward pass + contact Jacobians", "backward pass + L^T D L", "free velocity", "contact rows (Z, c)",
          "PGS sweeps", "back-substitution + integrate", "PD torque", "kernel outputs", "(count)", "(count)", "(unused)",
          "self-collision prepass"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--num-envs", type=int, default=4096)
    ap.add_argument("--trimesh", action="store_true", help="terrainType=trimesh (the lane team's TERR form)")
    a = ap.parse_args()
    import torch
    import isaacgymenvs
    from isaacgymenv_amd.isaacgym import _lib
    L = _lib.lib()
    env = isaacgymenvs.make(seed=42, task="AnymalTerrain", num_envs=a.num_envs, sim_device="cuda:0",
                            rl_device="cuda:0", headless=True, force_render=False,
                            overrides=["task.env.terrain.terrainType=trimesh"] if a.trimesh else [])
    N, A = env.num_envs, env.num_actions
    pool = torch.empty((64, N, A), device="cuda:0").uniform_(-1, 1)
    for i in range(a.warmup):
        env.step(pool[i % 64])
    buf = (C.c_ulonglong * 64)()
    assert L.gs_debug_phase_cycles(buf, 64, 1) == 0, "not the profiling build"
    for i in range(a.steps):
        env.step(pool[i % 64])
    assert L.gs_debug_phase_cycles(buf, 64, 1) == 0
    waves = (N * 4 + 63) // 64
    substeps = 5
    per = [buf[i] / (a.steps * waves) for i in range(16)]
    total = sum(per[:8]) + per[11]
    print(f"cycles per launch per wave (s_memtime), {waves} waves, {a.steps} launches:")
    for i, name in enumerate(PHASES):
        if name.startswith("("):
            continue
        print(f"  {name:36s} {per[i]:10.0f}  {100 * per[i] / total:5.1f} %")
    print(f"  {'total':36s} {total:10.0f}")
    print(f"chain contacts executed per wave per PGS sweep: {per[8] / (substeps * 5):.2f} of 12")
    print(f"root contacts executed per wave per PGS sweep:  {per[9] / (substeps * 5):.2f} of 2")
    print(f"self-collision narrowphase entered per wave per substep: {buf[12] / (a.steps * waves * substeps):.4f}")
    hist = [buf[16 + i] for i in range(16)]
    print("waves by launch total (25k-cycle bins):", " ".join(f"{25 * i}k:{h}" for i, h in enumerate(hist) if h))
    if buf[48]:
        ns = buf[48]
        print(f"slow waves (> 250k cycles): {ns}; their mean phases:")
        for i, name in enumerate(PHASES):
            if not name.startswith("("):
                print(f"  {name:36s} {buf[32 + i] / ns:10.0f}")
        print(f"  PGS chain contacts per slow wave: {buf[32 + 8] / ns:.1f}")
    if a.trimesh:
        w = a.steps * waves
        print(f"mesh queries (inside the forward pass): may_contact culls {buf[50] / w:.0f} cycles per wave per launch, "
              f"the scans {buf[51] / w:.0f}; queries scanned per wave per substep {buf[52] / (w * substeps):.1f}")
    if buf[12]:
        print(f"self-collision narrowphase cycles per entry: {buf[13] / buf[12]:.0f}, of which the near pairs' "
              f"contacts in their lanes {buf[14] / buf[12]:.0f} (the rest: ranking, staging, pool entries); lanes of "
              f"teams with a near pair per entry {buf[15] / buf[12]:.1f} of 64; lane 0's team near pairs per entry "
              f"{buf[10] / buf[12]:.2f}")


if __name__ == "__main__":
    main()
