"""Split-K weight-gradient GEMMs with the tile-major (S2H_GEMM_CFG=4096, GemmArgs16::dbg bit 16) and
the split-major XCD order of the (split, tile) pairs (default), per-launch time in graph replays
(tools/gemm_graph_bench.py) on the step's weight-gradient shapes.   GPU only.
    python tools/splitk_order_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402
from gemm_graph_bench import graph_time  # noqa: E402

from sam2_video.kernels import _lib, ops  # noqa: E402

# (N out, K in, rows): memory-attention FFN / projections over the 7 frames' rows, Hiera MLP / qkv
SHAPES = [(2048, 256, 93184), (256, 2048, 93184), (768, 256, 93184), (256, 256, 93184), (256, 64, 374192),
          (448, 112, 131072), (112, 448, 131072), (336, 112, 131072), (896, 224, 32768), (224, 896, 32768),
          (1792, 448, 8192), (448, 1792, 8192), (1344, 448, 14112)]


def main():
    bf = torch.bfloat16
    for N, K, R in SHAPES:
        dy = torch.randn(R, N, device="cuda", dtype=bf)
        x = torch.randn(R, K, device="cuda", dtype=bf)
        dw = torch.zeros(N, K, device="cuda")
        db = torch.zeros(N, device="cuda")
        row = f"wgrad {N:5d}x{K:5d} over {R:6d} rows |"
        res = []
        for c, nm in ((4096, "tile-major"), (0, "split-major")):
            _lib.lib().s2h_gemm_config(c)
            dw.zero_()
            t = graph_time(lambda: ops.linear_wgrad(dy, x, dw, db=db))
            res.append(dw.clone())
            row += f" {nm} {t:7.1f} us"
        _lib.lib().s2h_gemm_config(0)
        rel = float((res[0] - res[1]).abs().max() / (res[0].abs().max() + 1e-20))
        print(row + f" | max rel diff {rel:.1e}", flush=True)


if __name__ == "__main__":
    main()
