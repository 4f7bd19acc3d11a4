"""GPU time of the step's main GEMM shapes: libsam2hip (s2h_gemm: linear / dgrad / wgrad) against
torch.matmul (hipBLASLt) on the same operands, each timed as 20 launches in one captured HIP graph.
The library number is the attainable target for a tuned tile on the shape; the wgrad rows time
torch with a bf16 output (ours accumulates fp32).   GPU only:  python tools/gemm_vs_lib.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

from gemm_graph_bench import graph_time  # noqa: E402
from sam2_video.kernels import ops  # noqa: E402

# (kind, M, N, K): fwd Y[M,N] = X[M,K] W[N,K]^T; dgrad dX[M,K] = dY[M,N] W[N,K]; wgrad dW[N,K] = dY[M,N]^T X[M,K]
SHAPES = [("fwd", 13312, 2048, 256), ("fwd", 13312, 256, 2048), ("fwd", 13312, 256, 256), ("fwd", 13312, 768, 256),
          ("fwd", 13312, 128, 256), ("fwd", 13312, 1024, 256), ("fwd", 8192, 1792, 448), ("fwd", 131072, 448, 112),
          ("fwd", 32768, 896, 224), ("fwd", 14112, 1344, 448), ("fwd", 104, 256, 256), ("fwd", 13, 256, 256),
          ("dgrad", 93184, 2048, 256), ("dgrad", 93184, 256, 2048), ("dgrad", 93184, 256, 256),
          ("dgrad", 8192, 1792, 448), ("dgrad", 8192, 448, 1792),
          ("wgrad", 93184, 2048, 256), ("wgrad", 93184, 256, 2048), ("wgrad", 93184, 256, 256),
          ("wgrad", 8192, 1792, 448), ("wgrad", 374192, 256, 64)]


def main():
    bf = torch.bfloat16
    torch.manual_seed(0)
    print(f"{'kind':6s} {'M':>7s} {'N':>5s} {'K':>5s}   s2h_us  torch_us  s2h_TF  torch_TF", flush=True)
    for kind, M, N, K in SHAPES:
        fl = 2.0 * M * N * K
        if kind == "fwd":
            x = torch.randn(M, K, device="cuda", dtype=bf)
            w = torch.randn(N, K, device="cuda", dtype=bf) * 0.05
            b = torch.zeros(N, device="cuda")
            out = torch.empty(M, N, device="cuda", dtype=bf)
            ours = lambda: ops.linear(x, w, b, out=out)  # noqa: E731
            lib = lambda: torch.matmul(x, w.t())  # noqa: E731
        elif kind == "dgrad":
            dy = torch.randn(M, N, device="cuda", dtype=bf)
            w = torch.randn(N, K, device="cuda", dtype=bf) * 0.05
            dx = torch.empty(M, K, device="cuda", dtype=bf)
            ours = lambda: ops.linear_dgrad(dy, w, dx=dx)  # noqa: E731
            lib = lambda: torch.matmul(dy, w)  # noqa: E731
        else:
            dy = torch.randn(M, N, device="cuda", dtype=bf)
            x = torch.randn(M, K, device="cuda", dtype=bf)
            dw = torch.zeros(N, K, device="cuda")
            ours = lambda: ops.linear_wgrad(dy, x, dw)  # noqa: E731
            lib = lambda: torch.matmul(dy.t(), x)  # noqa: E731
        t0 = graph_time(ours)
        t1 = graph_time(lib)
        print(f"{kind:6s} {M:7d} {N:5d} {K:5d}  {t0:7.1f}  {t1:8.1f}  {fl / t0 / 1e6:6.0f}  {fl / t1 / 1e6:8.0f}",
              flush=True)


if __name__ == "__main__":
    main()
