"""Run one attention shape (fwd + bwd) repeatedly, for rocprofv3 counter passes.  GPU only.
  python tools/attn_one.py B H Lq Lk D [iters] [p_drop]"""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))
import torch  # noqa: E402

from sam2_video.kernels import ops  # noqa: E402

B, H, Lq, Lk, D = (int(v) for v in sys.argv[1:6])
iters = int(sys.argv[6]) if len(sys.argv) > 6 else 5
p = float(sys.argv[7]) if len(sys.argv) > 7 else 0.1
q = torch.randn(B, Lq, H, D, device="cuda").to(torch.bfloat16)
k = torch.randn(B, Lk, H, D, device="cuda").to(torch.bfloat16)
v = torch.randn(B, Lk, H, D, device="cuda").to(torch.bfloat16)
o, lse = torch.empty_like(q), torch.empty(B, H, Lq, device="cuda")
do = torch.randn_like(q)
dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
for _ in range(iters):
    ops.attn_fwd(q, k, v, o, lse, 1 / math.sqrt(D), p_drop=p, seed=3)
    ops.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, 1 / math.sqrt(D), p_drop=p, seed=3)
torch.cuda.synchronize()
print("done")
