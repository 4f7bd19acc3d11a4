"""Tiling sweep (s2h_gemm_config 1..10) of the step's largest GEMM shapes, with the epilogues the
step uses (FFN up: ReLU + dropout; its backward dgrad: ReLU mask from the output, 1/keep).
GPU only.   python tools/gemm_sweep.py [--iters 20]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))

import torch  # noqa: E402

from sam2_video.kernels import _lib, ops  # noqa: E402

CFGS = {1: "64", 2: "128", 3: "128ns3", 4: "256x128", 5: "256", 6: "128x256", 7: "128x64", 8: "64x128", 9: "64ns3",
        10: "64k32ns4"}


def timeit(fn, iters):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    bf = torch.bfloat16
    cases = []
    for M, N, K in ((13312, 2048, 256), (93184, 2048, 256), (13312, 256, 2048), (93184, 256, 2048), (13312, 256, 256),
                    (93184, 256, 256), (8192, 1792, 448), (131072, 448, 112)):
        x = torch.randn(M, K, device="cuda", dtype=bf)
        w = torch.randn(N, K, device="cuda", dtype=bf) * 0.05
        b = torch.zeros(N, device="cuda")
        out = torch.empty(M, N, device="cuda", dtype=bf)
        cases.append((f"fwd {M}x{N}x{K} relu+drop", 2.0 * M * N * K,
                      lambda x=x, w=w, b=b, out=out: ops.linear(x, w, b, act="relu", out=out, drop_p=0.1, seed=5)))
        cases.append((f"fwd {M}x{N}x{K} plain", 2.0 * M * N * K, lambda x=x, w=w, out=out: ops.linear(x, w, out=out)))
        wt = torch.randn(K, N, device="cuda", dtype=bf)
        h = torch.relu(torch.randn(M, N, device="cuda", dtype=bf))
        dx = torch.empty(M, N, device="cuda", dtype=bf)
        cases.append((f"dgrad {M}x{N}x{K} relu-mask", 2.0 * M * N * K,
                      lambda x=x, wt=wt, h=h, dx=dx: ops.linear_dgrad(x, wt, dx=dx, pre=h, act="relu", alpha=1.1)))
    for name, fl, fn in cases:
        row = f"{name:34s}"
        for c in [0] + list(CFGS):
            _lib.lib().s2h_gemm_config(c)
            try:
                t = timeit(fn, a.iters)
                row += f" {CFGS.get(c, 'auto')}:{t * 1e3:.0f}us/{fl / t / 1e9:.0f}"
            except Exception as e:  # noqa: BLE001
                row += f" {CFGS.get(c, 'auto')}:ERR"
        _lib.lib().s2h_gemm_config(0)
        print(row, flush=True)


if __name__ == "__main__":
    main()
