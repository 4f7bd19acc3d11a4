"""Weight-gradient GEMM (dW[N, K] += dY[rows, N]^T X[rows, K], split-K fp32 atomics into the
gradient arena) per-launch time per tiling on the step's shapes (graph replays,
tools/gemm_graph_bench.py).   GPU only.   python tools/wgrad_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402
from gemm_graph_bench import graph_time  # noqa: E402

from sam2_video.kernels import _lib, ops  # noqa: E402

# (N out, K in, rows)
SHAPES = [(256, 256, 93184), (2048, 256, 93184), (256, 2048, 93184), (768, 256, 93184), (256, 64, 374192),
          (1792, 448, 8192), (448, 1792, 8192), (1344, 448, 14112), (448, 448, 14112), (256, 256, 13312)]
CFGS = ((7, "128x64"), (0, "auto"), (1, "64"), (2, "128"), (6, "128x256"), (4, "256x128"))


def main():
    bf = torch.bfloat16
    for N, K, R in SHAPES:
        dy = torch.randn(R, N, device="cuda", dtype=bf)
        x = torch.randn(R, K, device="cuda", dtype=bf)
        dw = torch.zeros(N, K, device="cuda")
        db = torch.zeros(N, device="cuda")
        row = f"wgrad {N}x{K} over {R} |"
        for c, nm in CFGS:
            _lib.lib().s2h_gemm_config(c)
            t = graph_time(lambda: ops.linear_wgrad(dy, x, dw, db=db))
            row += f" {nm} {t:6.1f}"
        _lib.lib().s2h_gemm_config(0)
        print(row, flush=True)


if __name__ == "__main__":
    main()
