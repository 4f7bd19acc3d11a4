"""Calibration sweep of the deterministic weight-gradient GEMM (csrc/gemm_wgrad.hip): per step shape,
graph-replayed time of every tile x a range of split counts (s2h_wgrad_force), against the cost
model's own choice.   GPU only.   python tools/wgrad_sweep.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402
from gemm_graph_bench import graph_time  # noqa: E402

from sam2_video.kernels import _lib, ops  # noqa: E402

from wgrad_bench import SHAPES  # noqa: E402

TILES = ["256x256", "256x128", "128x256", "128x128", "256x64", "64x256"]


def main():
    bf = torch.bfloat16
    ops.wgrad_workspace("cuda")
    h = _lib.lib()
    for N, K, R in SHAPES:
        dy = torch.randn(R, N, device="cuda", dtype=bf)
        x = torch.randn(R, K, device="cuda", dtype=bf)
        dw = torch.zeros(N, K, device="cuda")
        db = torch.zeros(N, device="cuda")
        h.s2h_wgrad_force(-1, 0)
        auto = graph_time(lambda: ops.linear_wgrad(dy, x, dw, db=db))
        print(f"wgrad {N}x{K} over {R}: model {auto:6.1f} us", flush=True)
        for t, name in enumerate(TILES):
            row = f"    {name:8s}"
            for s in (4, 8, 16, 32, 64, 128, 256):
                if s > max(1, R // 512):
                    break
                h.s2h_wgrad_force(t, s)
                row += f" s{s}:{graph_time(lambda: ops.linear_wgrad(dy, x, dw, db=db)):6.1f}"
            print(row, flush=True)
        h.s2h_wgrad_force(-1, 0)


if __name__ == "__main__":
    main()
