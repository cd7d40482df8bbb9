"""Diagnose the TERR (mesh-contact) kernel vs the oracle: per-column error, self-collision on/off,
host backend beside the GPU.  python tools/probes/terr_diag.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle.oracle import OracleSim  # noqa: E402
from tests import helpers as H  # noqa: E402
from tests.test_terrain_gpu import _terrain_states  # noqa: E402


def run(ter, n, sc, host):
    art, flat = H.anymal()
    flat["self_collide"] = sc
    params = dict(H.ANYMAL_PARAMS, has_ground=0)
    root, dof, tau, mu = _terrain_states(n, ter, 2)
    gym, sim = H.make_gpu_sim("anymal", n, params, terrain=ter, host=host, self_collide=sc)
    H.load_state_into(sim, root, dof, mu)
    sim.dof_force.copy_(torch.from_numpy(tau.astype(np.float32).reshape(-1)).to(sim.dof_force.device))
    osim = OracleSim(flat, params, terrain=ter["oracle"])
    r, d = root.copy(), dof.copy()
    cf = np.zeros((n, flat["nb"], 3))
    gym.simulate(sim)
    osim.simulate(r, d, np.ascontiguousarray(tau), mu, cf)
    if not host:
        torch.cuda.synchronize()
    g_root, g_dof = H.read_state(sim, 12)
    err = np.abs(g_root - r)
    print(f"sc={sc} host={host}: root err per column max", np.array2string(err.max(0), precision=2),
          " envs off>2e-5 in pose:", int((err[:, :7] > 2e-5).any(1).sum()),
          " dof pos max", float(np.abs(g_dof[:, :, 0] - d[:, :, 0]).max()))
    bad = np.where((err[:, :7] > 2e-5).any(1))[0][:5]
    for i in bad:
        print("   env", i, "gpu", np.round(g_root[i, :7], 5), "oracle", np.round(r[i, :7], 5))


if __name__ == "__main__":
    ter = H.rough_terrain(seed=5)
    for sc in (0, 1):
        for host in ((True,) if not __import__("torch").cuda.is_available() else (True, False)):
            run(ter, 128, sc, host)
