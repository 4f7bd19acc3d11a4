"""True GPU time of small / medium GEMM launches: 20 launches captured in one HIP graph and
replayed (eager timing of one launch is bounded by the host's ctypes + launch cost, ~12 us).
GPU only.   python tools/gemm_graph_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))

import torch  # noqa: E402

from sam2_video.kernels import _lib, ops  # noqa: E402

CFGS = {0: "auto", 1: "64", 2: "128", 7: "128x64", 8: "64x128", 9: "64ns3", 10: "64k32ns4"}
SHAPES = [(13312, 256, 256), (13312, 128, 256), (13312, 768, 256), (13312, 1024, 256), (13312, 2048, 256),
          (13312, 256, 2048), (104, 256, 256), (104, 256, 2048), (104, 2048, 256), (13, 256, 256),
          (8192, 256, 896), (93548, 256, 64)]


def graph_time(fn, n=20, reps=5):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / (n * reps) * 1e3  # us per launch


_SCRUB = None


def graph_time_cold(fn, n=8, reps=3):
    """per-launch GPU time with the caches cold: every launch follows a pass over a 512 MB buffer
    (evicts the XCD L2s and the 256 MB Infinity Cache, like the step's operands that were written
    long before); the scrub's own time, captured alone, is subtracted"""
    global _SCRUB
    if _SCRUB is None:
        _SCRUB = torch.empty(128 * 2**20, device="cuda", dtype=torch.float32)
    scrub = lambda: _SCRUB.mul_(0.5)  # noqa: E731
    both = graph_time(lambda: (scrub(), fn()), n=n, reps=reps)
    alone = graph_time(scrub, n=n, reps=reps)
    return both - alone


def main():
    bf = torch.bfloat16
    for M, N, K in SHAPES:
        x = torch.randn(M, K, device="cuda", dtype=bf)
        w = torch.randn(N, K, device="cuda", dtype=bf) * 0.05
        b = torch.zeros(N, device="cuda")
        r = torch.randn(M, N, device="cuda", dtype=bf)
        out = torch.empty(M, N, device="cuda", dtype=bf)
        row = f"{M}x{N}x{K:<6}"
        for c, nm in CFGS.items():
            _lib.lib().s2h_gemm_config(c)
            t = graph_time(lambda: ops.linear(x, w, b, out=out))
            t2 = graph_time(lambda: ops.linear(x, w, b, out=out, residual=r, drop_p=0.1, seed=3))
            row += f"  {nm}:{t:5.1f}/{t2:5.1f}"
        _lib.lib().s2h_gemm_config(0)
        print(row, flush=True)


if __name__ == "__main__":
    main()
