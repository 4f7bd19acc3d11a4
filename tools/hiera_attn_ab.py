"""Hiera attention backward (flash path, head dim 56 in the 64 image) on the B+ 512^2 8-frame
shapes -- stage-3 14x14 windows and the global blocks -- inside captured graphs.  Run once per
build: S2H_LIB_PATH=<lib> python tools/hiera_attn_ab.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402
from gemm_graph_bench import graph_time  # noqa: E402

from sam2_video.kernels import ops  # noqa: E402

SHAPES = [(72 * 8, 196, 8, 56), (8, 1024, 8, 56), (32, 1024, 16, 56)]  # (B, L, H, D)


def main():
    row = os.path.basename(os.environ.get("S2H_LIB_PATH", "default")) + " |"
    for B, L, H, D in SHAPES:
        q, k, v, do = (torch.randn(B, L, H, D, device="cuda").to(torch.bfloat16) for _ in range(4))
        o = torch.empty_like(q)
        lse = torch.empty(B, H, L, device="cuda")
        ops.attn_fwd(q, k, v, o, lse, D ** -0.5)
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        t = graph_time(lambda: ops.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, D ** -0.5), n=10)
        row += f" {B}x{L}x{H}: bwd {t:6.1f} us |"
    print(row, flush=True)


if __name__ == "__main__":
    main()
