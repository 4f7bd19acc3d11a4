"""Run LayerNorm forward (fused add) + backward on one shape repeatedly (rocprofv3 kernel traces).
  python tools/ln_one.py rows C [iters]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))
import torch  # noqa: E402

from sam2_video.kernels import ops  # noqa: E402

rows, C = int(sys.argv[1]), int(sys.argv[2])
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 20
x = torch.randn(rows, C, device="cuda").to(torch.bfloat16)
r = torch.randn(rows, C, device="cuda").to(torch.bfloat16)
g = torch.randn(C, device="cuda")
b = torch.randn(C, device="cuda")
xs = torch.empty_like(x)
dy = torch.randn_like(x)
dg, db = torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda")
for _ in range(iters):
    y, mean, rstd = ops.layernorm_fwd(x, g, b, 1e-5, add=r, xsum=xs)
    ops.layernorm_bwd(xs, dy, g, mean, rstd, dgamma=dg, dbeta=db, dres=dy)
torch.cuda.synchronize()
print("done")
