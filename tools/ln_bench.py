"""Per-launch GPU time of the LayerNorm forward / backward on the step's shapes (graph replays,
tools/gemm_graph_bench.py).  Run once per build: S2H_LIB_PATH=<lib> python tools/ln_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402
from gemm_graph_bench import graph_time  # noqa: E402

from sam2_video.kernels import ops  # noqa: E402

SHAPES = [(13312, 256), (131072, 112), (32768, 224), (8192, 448), (2048, 896), (93184, 256)]


def main():
    row = os.path.basename(os.environ.get("S2H_LIB_PATH", "default")) + " |"
    for R, C in SHAPES:
        x = torch.randn(R, C, device="cuda").to(torch.bfloat16)
        dy = torch.randn_like(x)
        g, b = torch.randn(C, device="cuda"), torch.randn(C, device="cuda")
        y, mu, rs = ops.layernorm_fwd(x, g, b, 1e-6)
        dg, db = torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda")
        dx = torch.empty_like(x)
        tf = graph_time(lambda: ops.layernorm_fwd(x, g, b, 1e-6, y=y))
        tb = graph_time(lambda: ops.layernorm_bwd(x, dy, g, mu, rs, dx=dx, dgamma=dg, dbeta=db))
        row += f" {R}x{C}: fwd {tf:5.1f} bwd {tb:5.1f} |"
    print(row, flush=True)


if __name__ == "__main__":
    main()
