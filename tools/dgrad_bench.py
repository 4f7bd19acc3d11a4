"""dgrad (dX = dY W: A K-contiguous, B row-contiguous) per-launch time per tiling on the step's
shapes (graph replays, tools/gemm_graph_bench.py).   GPU only.   python tools/dgrad_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402
from gemm_graph_bench import graph_time  # noqa: E402

from sam2_video.kernels import _lib, ops  # noqa: E402

# (rows M, layer out N, layer in K): dX [M, K] = dY [M, N] W [N, K]
SHAPES = [(93184, 2048, 256), (8192, 1792, 448), (93184, 256, 2048), (93184, 256, 256), (93184, 256, 768), (131072, 448, 112), (32768, 672, 224),
          (8192, 448, 1792), (13312, 256, 256), (106496, 256, 64)]
CFGS = ((7, "128x64"), (0, "auto"), (1, "64"), (11, "128x64k32ns3"), (2, "128"))


def main():
    bf = torch.bfloat16
    for M, N, K in SHAPES:
        dy = torch.randn(M, N, device="cuda", dtype=bf)
        w = torch.randn(N, K, device="cuda", dtype=bf) * 0.05
        dx = torch.empty(M, K, device="cuda", dtype=bf)
        row = f"dgrad {M}x{K} (K={N}) |"
        for c, nm in CFGS:
            _lib.lib().s2h_gemm_config(c)
            t = graph_time(lambda: ops.linear_dgrad(dy, w, dx=dx))
            row += f" {nm} {t:6.1f}"
        _lib.lib().s2h_gemm_config(0)
        print(row, flush=True)


if __name__ == "__main__":
    main()
