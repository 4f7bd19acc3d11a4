"""Where the time of the step's short-K forward GEMMs goes (13312 rows x N x 256, the memory
attention's projections / FFN): cold-cache graph time per tiling, and for the automatic tiling the
measurement-only ablations of s2h_gemm_config bits 8+ (1 skip the epilogue stores, 2 skip the MFMAs,
4 skip the operand DMA) -- each epilogue the step uses (bias; bias + residual; ReLU + dropout).
    python tools/gemm_breakdown.py [--hot] [--cfgs 0,1,9,18]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import argparse  # noqa: E402

import torch  # noqa: E402

from gemm_graph_bench import graph_time, graph_time_cold  # noqa: E402
from sam2_video.kernels import _lib, ops  # noqa: E402

SHAPES = [(13312, 256, 256), (13312, 2048, 256), (13312, 768, 256), (13312, 128, 256), (13312, 256, 2048),
          (93184, 256, 256)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hot", action="store_true")
    ap.add_argument("--cfgs", default="0,1,20,18,23,7,21,11,22,13,24")
    ap.add_argument("--ablate", type=int, default=1)
    ap.add_argument("--shapes", type=int, default=99, help="first N shapes only")
    a = ap.parse_args()
    gt = graph_time if a.hot else graph_time_cold
    bf = torch.bfloat16
    torch.manual_seed(0)
    cfgs = [int(c) for c in a.cfgs.split(",")]
    L = _lib.lib()
    for M, N, K in SHAPES[:a.shapes]:
        x = torch.randn(M, K, device="cuda", dtype=bf)
        w = torch.randn(N, K, device="cuda", dtype=bf) * 0.05
        b = torch.zeros(N, device="cuda")
        r = torch.randn(M, N, device="cuda", dtype=bf)
        out = torch.empty(M, N, device="cuda", dtype=bf)
        epis = {"bias": lambda: ops.linear(x, w, b, out=out),
                "res": lambda: ops.linear(x, w, b, out=out, residual=r),
                "reludrop": lambda: ops.linear(x, w, b, act="relu", out=out, drop_p=0.1, seed=3)}
        for en, fn in epis.items():
            row = f"{M}x{N}x{K:<5} {en:9s}"
            for c in cfgs:
                L.s2h_gemm_config(c)
                row += f" c{c}:{gt(fn):6.1f}"
            if a.ablate:
                for d, nm in ((1, "nostore"), (2, "nomfma"), (4, "nodma"), (6, "storeonly"), (7, "skeleton"),
                              (8, "plainst"), (14, "storeonly_plain")):
                    L.s2h_gemm_config(d << 8)
                    row += f" {nm}:{gt(fn):6.1f}"
            L.s2h_gemm_config(0)
            row += f" hipblaslt:{gt(lambda: torch.matmul(x, w.t())):6.1f}"
            print(row, flush=True)


if __name__ == "__main__":
    main()
