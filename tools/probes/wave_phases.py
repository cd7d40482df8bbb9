"""Phase cycles of the wave-assisted UsefulHound simulate kernel (profiling build):
    python -m isaacgymenv_amd.build --prof && GS_LIBGYMSIM=libgymsim_prof.so python tools/probes/wave_phases.py
Prints per-wave s_memtime cycles per substep launch of: publish, terrain queries, pair broadphase, pair
narrowphase, env-lane substep (gs_physics_impl.h GS_WPROF)."""
import ctypes as C
import json
import os
import sys

os.environ.setdefault("GS_LIBGYMSIM", "libgymsim_prof.so")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

NAMES = ["publish", "terrain queries", "pair broadphase", "pair narrowphase", "env-lane substep"]


def main():
    import torch
    import isaacgymenvs
    from isaacgymenv_amd.isaacgym import _lib
    L = _lib.lib()
    fn = getattr(L, "gs_debug_wave_cycles_Topo_hound_0")
    fn.argtypes = [C.POINTER(C.c_ulonglong), C.c_int, C.c_int]
    env = isaacgymenvs.make(seed=42, task="UsefulHound", num_envs=4096, sim_device="cuda:0", rl_device="cuda:0",
                            graphics_device_id=-1, headless=True, force_render=False)
    act = torch.empty((env.num_envs, env.num_actions), device="cuda:0").uniform_(-1, 1)
    env.reset()
    for _ in range(3):
        env.step(act)
    buf = (C.c_ulonglong * 16)()
    assert fn(buf, 16, 1) == 0
    launches = 10
    for _ in range(launches):
        env.gym.simulate(env.sim)
    assert fn(buf, 16, 1) == 0
    waves = buf[8]
    per = {NAMES[i]: buf[i] / max(waves, 1) for i in range(5)}
    tot = sum(per.values())
    out = {"kernel": "k_simulate_wave<Topo_hound, false, true>", "waves": waves, "launches": launches,
           "cycles_per_wave_launch": per, "share": {k: v / tot for k, v in per.items()}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
