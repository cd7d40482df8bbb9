"""Per-layer timing of the PPO update's hidden layers: the rl_linear MFMA kernels vs the torch / hipBLASLt statements
they replace (AnymalTerrainPPO shapes, 16384-row minibatch, fp16).  HIP events, 50 repetitions after warm-up.

    python tools/probes/linear_probe.py [--out gpurun_out/linear_probe.json]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from isaacgymenv_amd.rl import gae, network  # noqa: E402


def timed(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--rows", type=int, default=16384)
    ap.add_argument("--splits-sweep", action="store_true", help="also time dW + finish at 8 ... 128 row blocks")
    a = ap.parse_args()
    M = a.rows
    h = torch.float16
    res = []
    for K, N in ((188, 512), (512, 256), (256, 128)):
        x = torch.randn(M, K, device="cuda").to(h)
        w = (torch.randn(N, K, device="cuda") * 0.05).to(h)
        b = (torch.randn(N, device="cuda") * 0.05).to(h)
        y = torch.empty(M, N, dtype=h, device="cuda")
        dy = torch.randn(M, N, device="cuda").to(h)
        wt = torch.empty(K, N, dtype=h, device="cuda")
        dx = torch.empty(M, K, dtype=h, device="cuda")
        splits = network._splits(M, (N // 128) * ((K + 127) // 128))
        part = torch.empty(splits, N * K + N, device="cuda")
        gacc = torch.zeros(N * K + N, device="cuda")
        r = {"M": M, "K": K, "N": N, "splits": splits}
        r["fwd_mfma"] = timed(lambda: gae.linear_fwd(x, w, b, True, y))
        r["fwd_torch"] = timed(lambda: torch.nn.functional.elu(torch.nn.functional.linear(x, w, b)))
        r["transpose"] = timed(lambda: gae.linear_transpose(w, wt))
        if K % 128 == 0:
            r["dx_mfma"] = timed(lambda: gae.linear_bwd(dy, y, x, w, dx, splits, None, None))
        r["dw_mfma"] = timed(lambda: gae.linear_bwd(dy, y, x, None, None, splits, part, part[:, N * K:], N * K + N))
        r["accum"] = timed(lambda: gae.splitk_accum(part, gacc))
        if a.splits_sweep:
            for S in (8, 16, 32, 64, 128):
                if M % (S * 64):
                    continue
                pt = torch.empty(S, N * K + N, device="cuda")
                r[f"dw_s{S}"] = timed(lambda: gae.linear_bwd(dy, y, x, None, None, S, pt, pt[:, N * K:], N * K + N))
                r[f"acc_s{S}"] = timed(lambda: gae.splitk_accum(pt, gacc))

        def torch_bwd():
            dz = torch.ops.aten.elu_backward(dy, 1.0, 1.0, 1.0, True, y)
            if K % 128 == 0:
                dz @ w
            p = torch.bmm(dz.reshape(16, M // 16, N).transpose(1, 2), x.reshape(16, M // 16, K))
            p.sum(0, dtype=torch.float32)
            dz.sum(0, dtype=torch.float32)
        r["bwd_torch"] = timed(torch_bwd)
        r["bwd_mfma_total"] = r.get("dx_mfma", 0.0) + r["dw_mfma"] + r["accum"]
        flops = 2 * M * N * K
        r["fwd_mfma_tflops"] = flops / r["fwd_mfma"] / 1e6
        r["dw_mfma_tflops"] = flops / r["dw_mfma"] / 1e6
        print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
        res.append(r)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
