"""GEMM probe: every LDS-DMA tiling of libsam2hip's bf16 GEMM (s2h_gemm_config) on the training
step's shapes, checked against torch.matmul (hipBLASLt) and timed beside it.  GPU only.

  python tools/gemm_probe.py [--iters 20] [--cfgs 2,3,4,5,6]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))
import torch  # noqa: E402

from sam2_video.kernels import _lib, ops  # noqa: E402

CFG_NAMES = {1: "64", 2: "128", 3: "128s3", 4: "256x128", 5: "256", 6: "128x256", 7: "128x64", 8: "64x128", 9: "64s3",
             10: "64k32s4", 11: "128k32s4", 12: "128k32s5", 13: "256x128k32", 14: "256k32s4", 15: "128x64k32s6",
             16: "64k32s6", 17: "p64", 18: "p64s3", 19: "p128", 20: "p128x64", 21: "p64x128", 22: "p256",
             23: "p128s3"}
# (M, N, K, kind): fwd = x[M,K] @ w[N,K]^T ; dgrad = dy[M,K] @ w[K,N] ; wgrad = dy[K,M]^T @ x[K,N] (fp32 out)
SHAPES = [
    (13312, 2048, 256, "fwd"), (13312, 256, 2048, "fwd"), (13312, 768, 256, "fwd"), (13312, 256, 256, "fwd"),
    (13312, 2048, 256, "dgrad"), (13312, 256, 2048, "dgrad"), (13312, 256, 768, "dgrad"),
    (2048, 256, 13312, "wgrad"), (256, 2048, 13312, "wgrad"), (768, 256, 13312, "wgrad"),
    (8192, 1792, 448, "fwd"), (8192, 448, 1792, "fwd"), (14112, 1344, 448, "fwd"), (8192, 1792, 448, "dgrad"),
    (131072, 448, 112, "fwd"), (131072, 112, 448, "dgrad"), (32768, 896, 224, "fwd"),
    (93548, 256, 64, "fwd"), (4096, 4096, 4096, "fwd"),
]


def timeit(fn, iters):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--cfgs", default="0,2,3,4,5,6")
    a = ap.parse_args()
    cfgs = [int(c) for c in a.cfgs.split(",")]
    bf = torch.bfloat16
    head = "".join(f"{('auto' if c == 0 else CFG_NAMES[c]):>10s}" for c in cfgs)
    print(f"{'shape':24s} {'kind':6s}{head} {'hipblaslt':>10s}   (us; TF/s of best)", flush=True)
    for M, N, K, kind in SHAPES:
        fl = 2.0 * M * N * K
        if kind == "fwd":
            x = torch.randn(M, K, device="cuda", dtype=bf)
            w = torch.randn(N, K, device="cuda", dtype=bf)
            out = torch.empty(M, N, device="cuda", dtype=bf)
            ours = lambda: ops.linear(x, w, out=out)  # noqa: E731
            ref = lambda: x @ w.t()  # noqa: E731
        elif kind == "dgrad":
            x = torch.randn(M, K, device="cuda", dtype=bf)
            w = torch.randn(K, N, device="cuda", dtype=bf)
            out = torch.empty(M, N, device="cuda", dtype=bf)
            ours = lambda: ops.linear_dgrad(x, w, dx=out)  # noqa: E731
            ref = lambda: x @ w  # noqa: E731
        else:
            x = torch.randn(K, M, device="cuda", dtype=bf)
            w = torch.randn(K, N, device="cuda", dtype=bf)
            out = torch.zeros(M, N, device="cuda")
            ours = lambda: ops.linear_wgrad(x, w, out, accumulate=False)  # noqa: E731
            ref = lambda: x.t() @ w  # noqa: E731
        r = ref().float()
        row = []
        for c in cfgs:
            _lib.lib().s2h_gemm_config(c)
            out.zero_()
            ours()
            err = ((out.float() - r).abs().max() / (r.abs().max() + 1e-6)).item()
            t = timeit(ours, a.iters)
            row.append((t, err))
        _lib.lib().s2h_gemm_config(0)
        tr = timeit(ref, a.iters)
        best = min(t for t, _ in row)
        cells = "".join(f"{t:9.1f}{'!' if e > 2e-2 else ' '}" for t, e in row)
        print(f"{M}x{N}x{K:<14} {kind:6s}{cells} {tr:9.1f}    {fl / best / 1e6:7.1f} vs {fl / tr / 1e6:7.1f}",
              flush=True)


if __name__ == "__main__":
    main()
