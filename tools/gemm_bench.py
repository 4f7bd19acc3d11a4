"""Microbenchmark of libsam2hip's bf16 GEMM on the training step's hot shapes, with
torch.matmul (hipBLASLt) on the same shapes as a yardstick.  GPU only.

  python tools/gemm_bench.py [--iters 20]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))

import torch  # noqa: E402

from sam2_video.kernels import ops  # noqa: E402

# (M, N, K, kind): fwd = x[M,K] @ w[N,K]^T ; dgrad = dy[M,K] @ w[K,N] ; wgrad = dy[K,M]^T @ x[K,N] (fp32 out)
SHAPES = [
    (13312, 2048, 256, "fwd"), (13312, 256, 2048, "fwd"), (13312, 768, 256, "fwd"), (13312, 256, 256, "fwd"),
    (13312, 128, 256, "fwd"), (13312, 1024, 256, "fwd"),
    (93184, 2048, 256, "dgrad"), (93184, 256, 2048, "dgrad"), (93184, 256, 256, "dgrad"),
    (2048, 256, 93184, "wgrad"), (256, 256, 93184, "wgrad"), (256, 2048, 93184, "wgrad"), (256, 64, 374192, "wgrad"),
    (1792, 448, 8192, "wgrad"), (448, 1792, 8192, "wgrad"),
    (8192, 1792, 448, "fwd"), (8192, 448, 1792, "fwd"), (14112, 1344, 448, "fwd"),
    (131072, 448, 112, "fwd"), (93548, 256, 64, "fwd"),
    (104, 256, 2048, "fwd"), (104, 256, 256, "fwd"), (104, 2048, 256, "fwd"), (13, 256, 256, "fwd"),
    (4096, 4096, 4096, "fwd"),
]


def timeit(fn, iters):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = "cuda"
    bf = torch.bfloat16
    print(f"{'shape':28s} {'kind':6s} {'ours ms':>9s} {'TF/s':>7s} {'torch ms':>9s} {'TF/s':>7s} {'maxrel':>8s}")
    for M, N, K, kind in SHAPES:
        fl = 2.0 * M * N * K
        if kind == "fwd":
            x = torch.randn(M, K, device=dev, dtype=bf)
            w = torch.randn(N, K, device=dev, dtype=bf)
            out = torch.empty(M, N, device=dev, dtype=bf)
            ours = lambda: ops.linear(x, w, out=out)  # noqa: E731
            ref = lambda: x @ w.t()  # noqa: E731
        elif kind == "dgrad":
            x = torch.randn(M, K, device=dev, dtype=bf)  # dy
            w = torch.randn(K, N, device=dev, dtype=bf)  # weight [out=K, in=N]
            out = torch.empty(M, N, device=dev, dtype=bf)
            ours = lambda: ops.linear_dgrad(x, w, dx=out)  # noqa: E731
            ref = lambda: x @ w  # noqa: E731
        else:
            x = torch.randn(K, M, device=dev, dtype=bf)  # dy [rows, out]
            w = torch.randn(K, N, device=dev, dtype=bf)  # x  [rows, in]
            out = torch.zeros(M, N, device=dev)
            ours = lambda: ops.linear_wgrad(x, w, out, accumulate=False)  # noqa: E731
            ref = lambda: x.t() @ w  # noqa: E731
        t_o = timeit(ours, a.iters)
        t_r = timeit(ref, a.iters)
        ours()
        r = ref().float()
        err = ((out.float() - r).abs().max() / (r.abs().max() + 1e-6)).item()
        print(f"{M}x{N}x{K:<16} {kind:6s} {t_o:9.4f} {fl / t_o / 1e9:7.1f} {t_r:9.4f} {fl / t_r / 1e9:7.1f} {err:8.1e}",
              flush=True)


if __name__ == "__main__":
    main()
