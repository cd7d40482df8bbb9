"""Per-layer time of the rollout's f32 act-forward layers (rl_linear_fwd_f32_g) at 4096 rows, K stage 32 vs 64
(RL_F32_KSTEP), by HIP events over 200 launches each.  GPU box: python tools/probes/f32_linear_probe.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    from isaacgymenv_amd.rl import gae
    M, G = 4096, 2
    layers = [(188, 512, 1), (512, 256, 2), (256, 128, 2)]  # (K, N, groups): layer 0 is one GEMM over 2 x 512
    out = {}
    for ks in ("32", "64", "auto"):
        if ks == "auto":
            os.environ.pop("RL_F32_KSTEP", None)
        else:
            os.environ["RL_F32_KSTEP"] = ks
        res = []
        for K, N, g in layers:
            x = torch.randn(M, K * (G if g > 1 else 1), device="cuda")
            w = torch.randn(G, N, K, device="cuda") * 0.05
            b = torch.randn(G, N, device="cuda")
            y = torch.empty(M, G * N, device="cuda")
            if g == 1:
                run = lambda: gae.linear_fwd_f32(x, K, K, w, G * N, b, True, y, G * N, M)  # noqa: E731
            else:
                run = lambda: gae.linear_fwd_f32(x, G * K, K, w, N, b, True, y, G * N, M, groups=G,  # noqa: E731
                                                 x_gstride=K, w_gstride=N * K, b_gstride=N, y_gstride=N)
            for _ in range(20):
                run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(200):
                run()
            e1.record()
            e1.synchronize()
            us = 1e3 * e0.elapsed_time(e1) / 200
            res.append({"K": K, "N": G * N, "us": round(us, 2), "tflops": round(2 * M * K * G * N / us / 1e6, 1)})
        out["ks_" + ks] = res
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
