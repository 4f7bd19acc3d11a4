"""Run one bf16 forward GEMM shape repeatedly (for rocprofv3 counter passes).  GPU only.
  python tools/gemm_one.py M N K [iters] [cfg]   (cfg: s2h_gemm_config tiling, 0 = automatic)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))
import torch  # noqa: E402

from sam2_video.kernels import _lib, ops  # noqa: E402

M, N, K = (int(a) for a in sys.argv[1:4])
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 5
if len(sys.argv) > 5:
    _lib.lib().s2h_gemm_config(int(sys.argv[5]))
x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(iters):
    ops.linear(x, w, out=out)
torch.cuda.synchronize()
print("done")
