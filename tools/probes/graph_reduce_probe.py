"""Which reductions survive HIP-graph replay?  Each op: eager result vs 5 replays of a capture."""
import torch

torch.manual_seed(0)
dev = "cuda"
cases = {
    "sum0_8192x32": (lambda x: x.sum(0), torch.randn(8192, 32, device=dev)),
    "sum0_8192x1": (lambda x: x.sum(0), torch.randn(8192, 1, device=dev)),
    "sum0_16384x512": (lambda x: x.sum(0), torch.randn(16384, 512, device=dev)),
    "sum0_16384x128": (lambda x: x.sum(0), torch.randn(16384, 128, device=dev)),
    "mean_8192": (lambda x: x.mean(), torch.randn(8192, device=dev)),
    "mean_1M": (lambda x: x.mean(), torch.randn(1 << 20, device=dev)),
    "sum1_8192x32": (lambda x: x.sum(1), torch.randn(8192, 32, device=dev)),
    "norm_2M": (lambda x: torch.linalg.vector_norm(x), torch.randn(2 << 20, device=dev)),
    "zeros_like": (lambda x: torch.zeros_like(x) + x, torch.randn(1000, device=dev)),
    "sum0_bias_ones_gemm": (lambda x: torch.ones(1, x.shape[0], device=dev) @ x, torch.randn(8192, 32, device=dev)),
}
for name, (fn, x) in cases.items():
    ref = fn(x).clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn(x)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        y = fn(x)
    diffs = []
    for k in range(5):
        g.replay()
        torch.cuda.synchronize()
        diffs.append((y - ref).abs().max().item())
    print(f"{name:24s} " + " ".join(f"{d:.3g}" for d in diffs), flush=True)
