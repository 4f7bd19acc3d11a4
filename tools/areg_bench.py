"""Short-K GEMMs: the automatic tiling against the A-in-registers tilings (gemm16a_kernel, cfg 29 =
64 x 64, 30 = 64 x 128), per-launch time in graph replays (tools/gemm_graph_bench.py), forward
(B K-contiguous) and input-gradient (B row-contiguous) layouts of the step's shapes, with the
step's epilogues (bias + ReLU + dropout; residual + dropout).   GPU only.
    python tools/areg_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402
from gemm_graph_bench import graph_time  # noqa: E402

from sam2_video.kernels import _lib, ops  # noqa: E402

# (M, N, K, B K-contiguous, epilogue)
SHAPES = [(13312, 256, 256, True, "res"), (13312, 768, 256, True, "bias"), (13312, 2048, 256, True, "relu"),
          (13312, 128, 256, True, "bias"), (13312, 256, 72, True, "res"), (93184, 256, 256, False, "plain"),
          (93184, 2048, 256, False, "plain"), (13312, 256, 128, True, "bias"), (104, 256, 256, True, "bias"),
          (8192, 448, 112, True, "bias"), (32768, 224, 224, True, "bias"), (131072, 112, 112, False, "plain")]


def main():
    bf = torch.bfloat16
    ops.rng_offset("cuda").fill_(3)
    for M, N, K, bkc, epi in SHAPES:
        a = torch.randn(M, K, device="cuda", dtype=bf)
        b = torch.randn(N, K, device="cuda", dtype=bf) if bkc else torch.randn(K, N, device="cuda", dtype=bf)
        c = torch.empty(M, N, device="cuda", dtype=bf)
        bias = torch.randn(N, device="cuda")
        res = torch.randn(M, N, device="cuda", dtype=bf)
        kw = dict(M=M, N=N, K=K, lda_m=K, lda_k=1, ldb_k=1 if bkc else N, ldb_n=K if bkc else 1, ldc=N)
        if epi == "res":
            kw.update(residual=res, ldr=N, drop_p=0.1, seed=5)
        elif epi == "relu":
            kw.update(bias=bias, act=1, drop_p=0.1, seed=5)
        elif epi == "bias":
            kw.update(bias=bias)
        row = f"{M:6d}x{N:5d}x{K:4d} {'fwd ' if bkc else 'dgrd'} {epi:5s} |"
        outs = []
        for cfg, nm in ((0, "auto"), (29, "areg64"), (30, "areg64x128")):
            _lib.lib().s2h_gemm_config(cfg)
            t = graph_time(lambda: ops.gemm(a, b, c, **kw))
            outs.append(c.clone())
            row += f" {nm} {t:7.1f}"
        _lib.lib().s2h_gemm_config(0)
        same = all(torch.equal(outs[0], o) for o in outs[1:])
        print(row + f" | identical {same}", flush=True)


if __name__ == "__main__":
    main()
