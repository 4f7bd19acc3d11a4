"""GPU time of the step's long-K / wide GEMM shapes under every LDS-DMA tiling (s2h_gemm_config),
20 launches per captured graph.  Which tiling reads the big operand once?   python tools/gemm_cfg_sweep.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import argparse  # noqa: E402

import torch  # noqa: E402

from gemm_graph_bench import graph_time, graph_time_cold  # noqa: E402
from sam2_video.kernels import _lib, ops  # noqa: E402

CFGS = {0: "auto", 1: "64", 2: "128", 7: "128x64", 11: "128x64k32", 16: "128k32", 14: "256x128w4k32",
        15: "256x128w4", 17: "256x64w4k32", 4: "256x128w8", 5: "256"}
SHAPES = [("fwd", 13312, 2048, 256), ("fwd", 13312, 1024, 256), ("fwd", 13312, 768, 256), ("fwd", 13312, 256, 256),
          ("fwd", 13312, 128, 256), ("fwd", 13312, 256, 2048), ("fwd", 8192, 1792, 448), ("fwd", 14112, 1344, 448),
          ("fwd", 32768, 896, 224), ("fwd", 131072, 448, 112), ("dgrad", 93184, 2048, 256), ("dgrad", 93184, 256, 2048),
          ("dgrad", 93184, 256, 256), ("dgrad", 8192, 448, 1792), ("dgrad", 8192, 1792, 448), ("dgrad", 131072, 112, 448)]


# weight gradients: dW [N_out, K_in] = dY^T X over `rows` (split-K regime); (kind, rows, N_out, K_in)
WGRAD = [("wgrad", 93184, 2048, 256), ("wgrad", 93184, 256, 2048), ("wgrad", 93184, 256, 256),
         ("wgrad", 93184, 768, 256), ("wgrad", 8192, 1792, 448), ("wgrad", 8192, 448, 1792),
         ("wgrad", 14112, 1344, 448), ("wgrad", 14112, 448, 448), ("wgrad", 374192, 256, 64),
         ("wgrad", 106496, 128, 256), ("wgrad", 32768, 896, 224), ("wgrad", 131072, 448, 112),
         ("wgrad", 131072, 112, 448), ("wgrad", 13312, 256, 256)]
# tiny-M forward GEMMs (per-object / per-token heads of the tracking loop)
TINY = [("fwd", 13, 256, 256), ("fwd", 104, 256, 256), ("fwd", 104, 128, 256), ("fwd", 104, 256, 2048),
        ("fwd", 104, 2048, 256), ("fwd", 13, 32, 256), ("fwd", 104, 256, 128), ("dgrad", 104, 256, 256),
        ("dgrad", 13, 256, 256)]
TCFGS = {0: "auto", 1: "64", 9: "64ns3", 18: "64ns4", 19: "64k32ns8", 10: "64k32ns4"}
WCFGS = {0: "auto", 1: "64", 9: "64ns3", 10: "64k32ns4", 7: "128x64", 13: "128x64ns3", 11: "128x64k32",
         12: "128x64k32ns4", 2: "128", 3: "128ns3", 16: "128k32"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--wgrad", action="store_true", help="sweep the weight-gradient shapes instead")
    ap.add_argument("--tiny", action="store_true", help="sweep the tiny-M head GEMMs instead")
    ap.add_argument("--cold", action="store_true", help="time every launch with cold caches (graph_time_cold)")
    args = ap.parse_args()
    bf = torch.bfloat16
    torch.manual_seed(0)
    cfgs = WCFGS if args.wgrad else TCFGS if args.tiny else CFGS
    gt = graph_time_cold if args.cold else graph_time
    for kind, M, N, K in (WGRAD if args.wgrad else TINY if args.tiny else SHAPES):
        if kind == "fwd":
            x = torch.randn(M, K, device="cuda", dtype=bf)
            w = torch.randn(N, K, device="cuda", dtype=bf) * 0.05
            out = torch.empty(M, N, device="cuda", dtype=bf)
            fn = lambda: ops.linear(x, w, None, out=out)  # noqa: E731
            lib = lambda: torch.matmul(x, w.t())  # noqa: E731
        elif kind == "wgrad":
            dy = torch.randn(M, N, device="cuda", dtype=bf)
            x = torch.randn(M, K, device="cuda", dtype=bf)
            dw = torch.zeros(N, K, device="cuda")
            fn = lambda: ops.linear_wgrad(dy, x, dw)  # noqa: E731
            lib = lambda: torch.matmul(dy.t(), x)  # noqa: E731
        else:
            dy = torch.randn(M, N, device="cuda", dtype=bf)
            w = torch.randn(N, K, device="cuda", dtype=bf) * 0.05
            dx = torch.empty(M, K, device="cuda", dtype=bf)
            fn = lambda: ops.linear_dgrad(dy, w, dx=dx)  # noqa: E731
            lib = lambda: torch.matmul(dy, w)  # noqa: E731
        row = f"{kind:5s} {M}x{N}x{K:<5d}"
        for c, nm in cfgs.items():
            _lib.lib().s2h_gemm_config(c)
            try:
                t = gt(fn)
                row += f"  {nm}:{t:6.1f}"
            except Exception as e:  # a tiling that does not take the shape
                row += f"  {nm}:err"
        _lib.lib().s2h_gemm_config(0)
        if kind == "wgrad":  # automatic tiling at other split-K targets (workgroups)
            for tgt in (256, 512, 1024, 1536):
                prev = _lib.lib().s2h_gemm_split_target(tgt)
                row += f"  auto@{tgt}:{gt(fn):6.1f}"
                _lib.lib().s2h_gemm_split_target(prev)
        row += f"  hipblaslt:{gt(lib):6.1f}"
        print(row, flush=True)


if __name__ == "__main__":
    main()
