"""Decoder-shape attention (token <-> image, head dim 16; token self-attention, head dim 32):
forward + backward launches for a kernel trace.  GPU only.   python tools/attn_small.py [iters]"""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))
import torch  # noqa: E402

from sam2_video.kernels import ops  # noqa: E402

it = int(sys.argv[1]) if len(sys.argv) > 1 else 5
for B, H, Lq, Lk, D in ((104, 8, 1024, 8, 16), (104, 8, 8, 1024, 16), (104, 8, 8, 8, 32)):
    q = torch.randn(B, Lq, H, D, device="cuda").to(torch.bfloat16)
    k = torch.randn(B, Lk, H, D, device="cuda").to(torch.bfloat16)
    v = torch.randn(B, Lk, H, D, device="cuda").to(torch.bfloat16)
    o = torch.empty_like(q)
    lse = torch.empty(B, H, Lq, device="cuda")
    do = torch.randn_like(q)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    for _ in range(it):
        ops.attn_fwd(q, k, v, o, lse, 1 / math.sqrt(D))
        ops.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, 1 / math.sqrt(D))
torch.cuda.synchronize()
print("done")
