"""Ablation timing of the LDS-DMA GEMM (measurement only; outputs are wrong when ablated):
full kernel, no epilogue stores, no MFMAs, neither -- per tiling.  GPU only."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))
import torch  # noqa: E402

from sam2_video.kernels import _lib, ops  # noqa: E402
from gemm_probe import timeit  # noqa: E402

bf = torch.bfloat16
CFGS = [int(c) for c in sys.argv[1].split(",")] if len(sys.argv) > 1 else [1, 2]
SHAPES = [(13312, 2048, 256), (13312, 256, 2048), (13312, 2048, 64), (4096, 4096, 4096)]
if len(sys.argv) > 2:
    SHAPES = [tuple(int(v) for v in s.split("x")) for s in sys.argv[2].split(",")]
for M, N, K in SHAPES:
    x = torch.randn(M, K, device="cuda", dtype=bf)
    w = torch.randn(N, K, device="cuda", dtype=bf)
    out = torch.empty(M, N, device="cuda", dtype=bf)
    for cfg in CFGS:
        row = []
        for dbg in (0, 1, 2, 3):
            _lib.lib().s2h_gemm_config(cfg | (dbg << 8))
            row.append(timeit(lambda: ops.linear(x, w, out=out), 20))
        _lib.lib().s2h_gemm_config(0)
        print(f"{M}x{N}x{K} cfg {cfg}: full {row[0]:7.1f}  no-store {row[1]:7.1f}  no-mfma {row[2]:7.1f}  "
              f"loads-only {row[3]:7.1f} us", flush=True)
