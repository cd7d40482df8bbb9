"""How often the self-contact pool cap and the deep-overlap skip act (measure the spec deviations of
DESIGN.md 3.12 instead of assuming them rare).

Rolls out AnymalTerrain and UsefulHound on the CPU pipeline (libgymsim host backend, the reference's random-action
usage, resets included), and every few steps hands the sim states to the fp64 oracle's self-contact narrowphase
twice: with the product's pool size (ANYmal 4, UsefulHound 8) and with 16 slots.  Reports per env-substep the
rate of envs whose contacts overflow the product pool, the contacts dropped, and the deep core overlaps skipped
(oracle_pair_stats).  Usage: python tools/pool_overflow_study.py [--envs 512] [--steps 300] [--every 10]"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def study(task, n, steps, every):
    import isaacgymenvs
    from isaacgymenv_amd.isaacgymenvs.tasks.base import vec_task
    from oracle import oracle as OO
    from tests import helpers as H
    vec_task.EXISTING_SIM = None
    env = isaacgymenvs.make(seed=42, task=task, num_envs=n, sim_device="cpu", rl_device="cpu", headless=True,
                            force_render=False)
    art, flat = H.anymal() if task == "AnymalTerrain" else H.hound()
    nd = flat["nd"]
    npool = int(flat["npool"])
    big = dict(flat)
    big["npool"] = 16
    o_prod, o_big = OO.OracleSim(flat, H.ANYMAL_PARAMS), OO.OracleSim(big, H.ANYMAL_PARAMS)
    lib = OO._lib(64)
    lib.oracle_pair_stats.restype = C.c_int
    st = (C.c_longlong * 7)()
    lib.oracle_pair_stats(st, 1)
    g = torch.Generator().manual_seed(3)
    samples = over = dropped = kept = deep = 0
    hist = np.zeros(17, np.int64)
    for t in range(steps):
        env.step(2 * torch.rand((n, env.num_actions), generator=g) - 1)
        if t % every:
            continue
        root, dof = H.read_state(env.sim, nd)
        mu = np.ascontiguousarray(env.sim.shape_mu.numpy().T[:, :flat["ns"]], dtype=np.float64)
        lib.oracle_pair_stats(st, 1)
        _, c_big = o_big.self_contacts(root, dof, mu)
        lib.oracle_pair_stats(st, 1)
        deep += st[5]
        _, c_prod = o_prod.self_contacts(root, dof, mu)
        samples += n
        over += int((c_big > npool).sum())
        dropped += int(np.maximum(c_big - npool, 0).sum())
        kept += int(c_prod.sum())
        hist += np.bincount(c_big, minlength=17)[:17]
    return dict(task=task, envs=n, env_steps=steps, sampled_env_states=samples, pool_slots=npool,
                envs_over_the_cap=over, over_rate=over / samples, contacts_dropped=dropped, contacts_kept=kept,
                dropped_per_kept=dropped / max(kept, 1), deep_overlaps_skipped=int(deep),
                deep_rate_per_env_state=deep / samples, contacts_per_env_histogram=hist.tolist())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=512)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--every", type=int, default=10)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    res = [study(t, a.envs, a.steps, a.every) for t in ("AnymalTerrain", "UsefulHound")]
    for r in res:
        print(json.dumps(r))
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
