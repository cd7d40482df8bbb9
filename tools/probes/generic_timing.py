"""Per-simulate time of the runtime-sized kernel (gs_generic.hip, kernel_variant 4) at 4096 envs, beside the
compiled kernels on the same robot (GPU box probe): Hound_new (no compiled topology), ANYmal forced generic vs the
lane-team / one-env-per-lane kernels (self-collision off, so all three run the same model).
    python tools/probes/generic_timing.py [--envs 4096]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def timed(kind, n, params, variant_env, states, drives=None):
    import torch
    from tests import helpers as H
    if variant_env:
        os.environ["GS_PHYSICS_KERNEL"] = variant_env
    else:
        os.environ.pop("GS_PHYSICS_KERNEL", None)
    gym, sim = H.make_gpu_sim(kind, n, params, drives=drives, self_collide=False)
    H.load_state_into(sim, *states)
    for _ in range(5):
        gym.simulate(sim)
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(20):
        gym.simulate(sim)
    e1.record(s)
    e1.synchronize()
    return {"robot": kind, "kernel": variant_env or "default", "kernel_variant": sim.kernel_variant,
            "envs": n, "ms_per_simulate": e0.elapsed_time(e1) / 20}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    a = ap.parse_args()
    from tests import helpers as H
    n = a.envs
    out = []
    root, dof, tau, mu = H.hound_new_states(n, seed=2, spread=0.2)
    root[:, 2] = 0.5
    out.append(timed("hound_new", n, dict(H.HOUND_PARAMS, solver_type=1), None, (root, dof, mu), H.HOUND_NEW_DRIVES))
    root, dof, tau, mu = H.anymal_states(n, seed=17)
    for v in ("generic", "lane", None):
        out.append(timed("anymal", n, dict(H.ANYMAL_PARAMS, solver_type=1), v, (root, dof, mu)))
    for o in out:
        print(json.dumps(o))


if __name__ == "__main__":
    main()
