"""GEMM probe: time of the bf16 forward GEMM vs K (fixed M, N) and vs N -- separates the
per-tile fixed cost (prologue latency, epilogue) from the per-K-step cost.  GPU only."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))
import torch  # noqa: E402

from sam2_video.kernels import ops  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


bf = torch.bfloat16
for M, N in ((13312, 2048), (13312, 256), (4096, 4096)):
    for K in (64, 128, 256, 512, 1024, 2048):
        x = torch.randn(M, K, device="cuda", dtype=bf)
        w = torch.randn(N, K, device="cuda", dtype=bf)
        out = torch.empty(M, N, device="cuda", dtype=bf)
        t = timeit(lambda: ops.linear(x, w, out=out))
        tt = timeit(lambda: x @ w.t())
        print(f"M {M} N {N} K {K:5d}: ours {t:8.1f} us {2 * M * N * K / t / 1e6:7.1f} TF/s | hipblaslt {tt:8.1f} us "
              f"{2 * M * N * K / tt / 1e6:7.1f} TF/s", flush=True)
