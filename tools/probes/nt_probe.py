"""Time the NT forward GEMM (rl_linear_fwd) on the learner's shapes and variants that isolate its parts:
ELU on / off, K = 188 / 192 / 64, N = 512 / 1024.  python tools/probes/nt_probe.py [out.json]"""
import json
import sys

import torch

from isaacgymenv_amd.rl import gae


def t_us(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000.0 / reps


res = []
M = 16384
for (N, K) in [(1024, 188), (1024, 192), (1024, 64), (512, 188), (512, 512), (256, 256)]:
    x = torch.randn(M, K, device="cuda").half()
    w = (0.05 * torch.randn(N, K, device="cuda")).half()
    b = torch.zeros(N, device="cuda").half()
    y = torch.empty(M, N, dtype=torch.float16, device="cuda")
    for act in (True, False):
        us = t_us(lambda: gae.linear_fwd(x, w, b, act, y))
        fl = 2.0 * M * N * K
        by = 2.0 * (M * K + N * K + M * N)
        res.append({"M": M, "N": N, "K": K, "elu": act, "us": us, "tflops": fl / us / 1e6, "gbs": by / us / 1e3})
        print(res[-1], flush=True)
    # the torch / hipBLASLt reference at the same shape
    us = t_us(lambda: torch.nn.functional.linear(x, w, b))
    res.append({"M": M, "N": N, "K": K, "torch_linear": True, "us": us})
    print(res[-1], flush=True)
if len(sys.argv) > 1:
    json.dump(res, open(sys.argv[1], "w"), indent=1)
