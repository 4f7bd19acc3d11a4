"""Microbenchmark of libsam2hip's attention on the memory-attention shapes (13 objects,
1 head of 256, Lq 1024, Lk 1024 / 1028*n) and a Hiera global shape, flash path on and off.
GPU only.   python tools/attn_bench.py [--iters 10] [--drop 0.1]
"""
import argparse
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))

import torch  # noqa: E402

from sam2_video.kernels import ops  # noqa: E402
from sam2_video.kernels._lib import lib  # noqa: E402

SHAPES = [(13, 1, 1024, 1024, 256), (13, 1, 1024, 3084, 256), (13, 1, 1024, 7196, 256), (8, 8, 1024, 1024, 64)]


def timeit(fn, iters):
    for _ in range(2):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def sweep_targets(a):
    for B, H, Lq, Lk, D in SHAPES:
        q = torch.randn(B, Lq, H, D, device="cuda").to(torch.bfloat16)
        k = torch.randn(B, Lk, H, D, device="cuda").to(torch.bfloat16)
        v = torch.randn(B, Lk, H, D, device="cuda").to(torch.bfloat16)
        o = torch.empty_like(q)
        lse = torch.empty(B, H, Lq, device="cuda")
        fl = 4.0 * B * H * Lq * Lk * D
        row = f"B{B} H{H} {Lq}x{Lk} d{D}:"
        for t in [int(x) for x in a.targets.split(",")]:
            lib().s2h_attn_config(1 | (t << 8))
            tf = timeit(lambda: ops.attn_fwd(q, k, v, o, lse, 1 / math.sqrt(D), p_drop=a.drop, seed=3), a.iters)
            row += f"  [{t}] {tf * 1e3:.0f} us {fl / tf / 1e9:.0f} TF/s"
        lib().s2h_attn_config(1)
        print(row, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--drop", type=float, default=0.1)
    ap.add_argument("--targets", default="", help="comma list of flash-forward split targets to sweep")
    a = ap.parse_args()
    if a.targets:
        return sweep_targets(a)
    for B, H, Lq, Lk, D in SHAPES:
        q = torch.randn(B, Lq, H, D, device="cuda").to(torch.bfloat16)
        k = torch.randn(B, Lk, H, D, device="cuda").to(torch.bfloat16)
        v = torch.randn(B, Lk, H, D, device="cuda").to(torch.bfloat16)
        o = torch.empty_like(q)
        lse = torch.empty(B, H, Lq, device="cuda")
        do = torch.randn_like(q)
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        sc = 1 / math.sqrt(D)
        fl = 4.0 * B * H * Lq * Lk * D
        row = f"B{B} H{H} {Lq}x{Lk} d{D} drop{a.drop}:"
        for flash in (1, 0):
            lib().s2h_attn_config(flash)
            tf = timeit(lambda: ops.attn_fwd(q, k, v, o, lse, sc, p_drop=a.drop, seed=3), a.iters)
            tb = timeit(lambda: ops.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, sc, p_drop=a.drop, seed=3), a.iters)
            row += (f"  [{'flash' if flash else 'generic'}] fwd {tf:.3f} ms {fl / tf / 1e9:.0f} TF/s"
                    f"  bwd {tb:.3f} ms {2.5 * fl / tb / 1e9:.0f} TF/s")
        lib().s2h_attn_config(1)
        print(row, flush=True)


if __name__ == "__main__":
    main()
