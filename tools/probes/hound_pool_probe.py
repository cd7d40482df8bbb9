"""Probe: self-contact pools of the Hound drives-test states (tests/test_drives.py _hound_vs_oracle, seed 9)
from the fp64 oracle, the host backend and (GPU) the device inline / split-record forms; then one simulate
per path, worst envs.  Usage: python tools/probes/hound_pool_probe.py [gpu] [env ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle.oracle import OracleSim  # noqa: E402
from tests import helpers as H  # noqa: E402
from tests.test_drives import DOF_MODE_EFFORT, DOF_MODE_POS, _run_oracle, _run_sim  # noqa: E402

gpu = "gpu" in sys.argv
envs = [int(a) for a in sys.argv[1:] if a.isdigit()] or [6, 11, 13]
n = 96
art, flat = H.hound()
root, dof, tau, mu = H.hound_states(n, seed=9)
rng = np.random.RandomState(4)
mode = np.full(18, DOF_MODE_EFFORT, dtype=np.int32)
mode[12:] = DOF_MODE_POS
kp = np.where(mode == DOF_MODE_POS, 300.0, 7000.0)
kd = np.where(mode == DOF_MODE_POS, 10.0, 50.0)
drives = (mode, kp, kd)
ptgt = rng.uniform(-1.0, 1.0, (n, 18))
vtgt = np.zeros((n, 18))

o_pool, o_cnt = OracleSim(flat, H.HOUND_PARAMS).self_contacts(root, dof, mu)
pools = {"oracle": (o_pool, o_cnt)}
for name, host in (("host", True),) + ((("gpu", False),) if gpu else ()):
    gym, sim = H.make_gpu_sim("hound", n, H.HOUND_PARAMS, host=host, drives=drives)
    H.load_state_into(sim, root, dof, mu)
    pools[name + "_inline"] = H.sim_self_contacts(sim, 0)
    if not host:
        pools[name + "_records"] = H.sim_self_contacts(sim, 1)


def diff(a, b):
    (pa, ca), (pb, cb) = a, b
    d = np.zeros(n)
    for e in range(n):
        if ca[e] != cb[e]:
            d[e] = np.inf
            continue
        k = ca[e]
        if k:
            d[e] = max(np.abs(pa[e, :k, 3:6] - pb[e, :k, 3:6]).max(), np.abs(pa[e, :k, :3] - pb[e, :k, :3]).max(),
                       np.abs(pa[e, :k, 6] - pb[e, :k, 6]).max())
    return d


for name in pools:
    if name == "oracle":
        continue
    d = diff(pools[name], pools["oracle"])
    w = np.argsort(-d)[:5]
    print(f"{name} vs oracle pool: count mismatches {int(np.isinf(d).sum())}, worst "
          + ", ".join(f"env {e}: {d[e]:.2e}" for e in w))
for e in envs:
    for name, (p, c) in pools.items():
        print(f"env {e} {name:>14s} count {c[e]}: bodies {[tuple(int(x) for x in p[e, i, 8:10]) for i in range(c[e])]}"
              f" sep {np.round(p[e, :c[e], 6], 5).tolist()}")

o_root, o_dof = _run_oracle(flat, H.HOUND_PARAMS, root, dof, tau, mu, ptgt, vtgt, drives, 1)
for name, host in (("host", True),) + ((("gpu", False),) if gpu else ()):
    gym, sim, (g_root, g_dof) = _run_sim("hound", n, H.HOUND_PARAMS, root, dof, tau, mu, ptgt, vtgt, drives, 1, host)
    eq = np.abs(g_dof[:, :, 0] - o_dof[:, :, 0]).max(1)
    w = np.argsort(-eq)[:5]
    print(f"{name} simulate vs oracle, dof pos: " + ", ".join(f"env {e}: {eq[e]:.2e}" for e in w))
    for e in envs:
        print(f"  env {e}: dq (1e-5) {np.round((g_dof[e, :, 0] - o_dof[e, :, 0]) * 1e5, 1).tolist()}")
