"""GPU time of the step's long-K / wide GEMM shapes under every LDS-DMA tiling (s2h_gemm_config),
20 launches per captured graph.  Which tiling reads the big operand once?   python tools/gemm_cfg_sweep.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

from gemm_graph_bench import graph_time  # noqa: E402
from sam2_video.kernels import _lib, ops  # noqa: E402

CFGS = {0: "auto", 1: "64", 2: "128", 4: "256x128", 5: "256", 6: "128x256", 7: "128x64", 13: "128x64ns3"}
SHAPES = [("dgrad", 93184, 2048, 256), ("dgrad", 93184, 256, 2048), ("dgrad", 93184, 256, 256),
          ("fwd", 13312, 2048, 256), ("fwd", 13312, 256, 2048), ("dgrad", 8192, 448, 1792), ("fwd", 8192, 1792, 448),
          ("dgrad", 8192, 1792, 448), ("fwd", 131072, 448, 112), ("dgrad", 131072, 112, 448)]


def main():
    bf = torch.bfloat16
    torch.manual_seed(0)
    for kind, M, N, K in SHAPES:
        if kind == "fwd":
            x = torch.randn(M, K, device="cuda", dtype=bf)
            w = torch.randn(N, K, device="cuda", dtype=bf) * 0.05
            out = torch.empty(M, N, device="cuda", dtype=bf)
            fn = lambda: ops.linear(x, w, None, out=out)  # noqa: E731
        else:
            dy = torch.randn(M, N, device="cuda", dtype=bf)
            w = torch.randn(N, K, device="cuda", dtype=bf) * 0.05
            dx = torch.empty(M, K, device="cuda", dtype=bf)
            fn = lambda: ops.linear_dgrad(dy, w, dx=dx)  # noqa: E731
        row = f"{kind:5s} {M}x{N}x{K:<5d}"
        for c, nm in CFGS.items():
            _lib.lib().s2h_gemm_config(c)
            try:
                t = graph_time(fn)
                row += f"  {nm}:{t:6.1f}"
            except Exception as e:  # a tiling that does not take the shape
                row += f"  {nm}:err"
        _lib.lib().s2h_gemm_config(0)
        print(row, flush=True)


if __name__ == "__main__":
    main()
