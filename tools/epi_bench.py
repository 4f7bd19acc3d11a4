"""GEMM epilogue-store experiments (graph-replay timing, tools/gemm_graph_bench.py): bf16 and
MX-fp8 GEMMs of the config-2 / config-5 shapes with plain vs non-temporal output stores and
with the stores skipped.   GPU only.   python tools/epi_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402
from gemm_graph_bench import graph_time  # noqa: E402

from sam2_video.kernels import _lib, ops  # noqa: E402

SHAPES = [(13312, 2048, 256), (13312, 256, 256), (13312, 768, 256), (8192, 1792, 448), (8192, 448, 1792),
          (93184, 2048, 256), (32768, 672, 224), (131072, 448, 112), (93184, 256, 2048), (104, 256, 256)]


def main():
    bf = torch.bfloat16
    for M, N, K in SHAPES:
        x = torch.randn(M, K, device="cuda", dtype=bf)
        w = torch.randn(N, K, device="cuda", dtype=bf) * 0.05
        b = torch.zeros(N, device="cuda")
        out = torch.empty(M, N, device="cuda", dtype=bf)
        row = f"{M}x{N}x{K:<6} MB out {M * N * 2 / 1e6:6.1f} |"
        for cfg, cn in ((0, "auto"), (1, "64"), (7, "128x64"), (11, "128x64k32ns3"), (2, "128"), (4, "256x128"),
                        (5, "256")):
            for dbg, nm in ((0, "nt"),):
                _lib.lib().s2h_gemm_config(cfg | (dbg << 8))
                t = graph_time(lambda: ops.linear(x, w, b, out=out))
                row += f" {cn}/{nm} {t:5.1f}"
            row += " |"
        _lib.lib().s2h_gemm_config(0)
        if K >= 128:
            x8, w8 = ops.mx8_quant(x), ops.mx8_quant(w)
            for dbg, nm in ((0, "nt"),):
                _lib.lib().s2h_mx8_config(dbg << 8)
                t = graph_time(lambda: ops.gemm_mx8(x8, w8, out, bias=b))
                row += f" mx8/{nm} {t:5.1f}"
            _lib.lib().s2h_mx8_config(0)
        print(row, flush=True)


if __name__ == "__main__":
    main()
