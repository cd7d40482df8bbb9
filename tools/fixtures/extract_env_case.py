"""Extract one env's inputs from a parity dump (tests/helpers.parity_dump, written on the GPU box under
gpurun_out/<run>/dump/) into a small fixture under tests/golden/.

    python tools/fixtures/extract_env_case.py gpurun_out/r05d/dump/hound4096.npz 680 tests/golden/hound_cylinder_ground_case.npz
"""
import sys

import numpy as np

src, env, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
z = np.load(src)
sl = slice(env, env + 1)
np.savez_compressed(out, **{k: z[k][sl] for k in ("root", "dof", "mu", "tau")}, source=np.array(f"{src} env {env}"))
print("wrote", out)
