import os, sys
HERE = os.path.dirname(os.path.abspath(__file__)); ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))
import torch, torch.nn.functional as F
from sam2_video.kernels import ops
from sam2_video.kernels.functional_sam import bicubic_matrix
C, bh, bw, h, w = 96, 7, 7, 64, 64
X = torch.randn(1, C, bh, bw)
ref = F.interpolate(X, size=(h, w), mode="bicubic")[0]
Ah, Aw = bicubic_matrix(bh, h, "cpu"), bicubic_matrix(bw, w, "cpu")
print("matrix form cpu err", (torch.einsum("ai,cij,bj->cab", Ah, X[0], Aw) - ref).abs().max().item())
Xd = X.cuda().reshape(C * bh, bw); Ahd, Awd = Ah.cuda(), Aw.cuda()
Y1 = torch.empty(C * bh, w, device="cuda")
ops.gemm(Xd, Awd, Y1, M=C * bh, N=w, K=bw, lda_m=bw, lda_k=1, ldb_k=1, ldb_n=bw, ldc=w)
print("Y1 err", (Y1.cpu() - X.reshape(C*bh, bw) @ Aw.t()).abs().max().item())
Y2 = torch.empty(C, h, w, device="cuda")
ops.gemm(Ahd, Y1, Y2, M=h, N=w, K=bh, lda_m=bh, lda_k=1, ldb_k=w, ldb_n=1, ldc=w, batch=C, sA=0, sB=bh * w, sC=h * w)
print("Y2 err", (Y2.cpu() - ref).abs().max().item())
