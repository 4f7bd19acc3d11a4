"""Per-launch GPU time of the MX-fp8 GEMM (s2h_gemm_mx8, every tiling) against the bf16 GEMM on
the config-5 projection / FFN shapes, plus the activation quantiser, inside captured graphs
(tools/gemm_graph_bench.py's timing).  Also a no-epilogue-store and a K-loop-only ablation
(s2h_mx8_config bits 8+).   GPU only.   python tools/mx8_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402
from gemm_graph_bench import graph_time  # noqa: E402

from sam2_video.kernels import _lib, ops  # noqa: E402

SHAPES = [(16384, 1792, 448), (16384, 448, 1792), (13312, 2048, 256), (13312, 256, 2048), (13312, 256, 256),
          (13312, 768, 256), (199680, 2048, 256), (65536, 672, 224), (4096, 2688, 896)]
MX = {1: "64x64", 2: "128x64", 3: "128x128"}


def main():
    bf = torch.bfloat16
    for M, N, K in SHAPES:
        x = torch.randn(M, K, device="cuda", dtype=bf)
        w = torch.randn(N, K, device="cuda", dtype=bf) * 0.05
        b = torch.zeros(N, device="cuda")
        out = torch.empty(M, N, device="cuda", dtype=bf)
        x8, w8 = ops.mx8_quant(x), ops.mx8_quant(w)
        fl = 2.0 * M * N * K
        t16 = graph_time(lambda: ops.linear(x, w, b, out=out))
        tq = graph_time(lambda: ops.mx8_quant(x, out=x8))
        row = f"{M}x{N}x{K:<6} bf16 {t16:6.1f} us ({fl / t16 / 1e6:5.0f} TF/s)  quant {tq:5.1f} us |"
        for c, nm in MX.items():
            _lib.lib().s2h_mx8_config(c)
            t = graph_time(lambda: ops.gemm_mx8(x8, w8, out, bias=b))
            row += f" {nm} {t:6.1f} ({fl / t / 1e6:5.0f})"
        for dbg, nm in ((1 << 8, "nostore"), (2 << 8, "nomfma"), (4 << 8, "nodma")):
            _lib.lib().s2h_mx8_config(3 | dbg)
            t = graph_time(lambda: ops.gemm_mx8(x8, w8, out, bias=b))
            row += f" {nm} {t:6.1f}"
        _lib.lib().s2h_mx8_config(0)
        print(row, flush=True)


if __name__ == "__main__":
    main()
