"""In-process A/B of the V-fold memory cross-attention backward as the training step runs it:
13 objects x 1024 queries against the 7 frames' packed memories (1028 n keys, n = 1..7), dropout
0.1 with the forward's keep bitmap, one frame-table launch (s2h_flash_bwd_frames_vfold).  Variants
by s2h_attn_config: 1 = current kernels (two-waves-per-SIMD dK), 3 = the one-wave-per-SIMD 32x32 dK
kernel.  Rounds interleave the variants.   GPU only:  python tools/vfold_ab.py [--iters 10] [--variants 1,3]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))

import torch  # noqa: E402

from sam2_video.kernels import ops  # noqa: E402
from sam2_video.kernels._lib import lib  # noqa: E402


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--drop", type=float, default=0.1)
    ap.add_argument("--variants", default="1,3")
    a = ap.parse_args()
    torch.manual_seed(0)
    B, Lq = 13, 1024
    lks = [1028 * n for n in range(1, 8)]
    F = len(lks)
    bf = torch.bfloat16
    sc = 256 ** -0.5
    q = (torch.randn(F * B, Lq, 1, 256, device="cuda") * 0.5).to(bf)
    rows = sum(B * lk for lk in lks)
    k = (torch.randn(rows, 1, 256, device="cuda") * 0.5).to(bf)
    m = torch.randn(rows, 1, 64, device="cuda").to(bf)
    u = torch.empty(F * B, Lq, 1, 72, device="cuda", dtype=bf)
    lse = torch.empty(F * B, 1, Lq, device="cuda")
    nw = [ops.keep_words(B, 1, Lq, lk) for lk in lks]
    koff = [sum(nw[:f]) for f in range(F)]
    keep = torch.zeros(sum(nw), device="cuda", dtype=torch.int32)
    krow, idx0, r, n = [], [], 0, 0
    for lk in lks:
        krow.append(r)
        idx0.append(n)
        r += B * lk
        n += B * Lq * lk
    for f, lk in enumerate(lks):
        sl = slice(f * B, (f + 1) * B)
        ops.attn_fwd_vfold(q[sl], k[krow[f]:krow[f] + B * lk].view(B, lk, 1, 256),
                           m[krow[f]:krow[f] + B * lk].view(B, lk, 1, 64), u[sl], lse[sl], sc, a.drop, 7,
                           idx0=idx0[f], keep=keep[koff[f]:koff[f] + nw[f]])
    du = torch.randn(F * B, Lq, 1, 72, device="cuda").to(bf)
    dq, dk = torch.empty_like(q), torch.empty_like(k)

    def bwd():
        ops.flash_bwd_frames_vfold(F, B, lks, krow, idx0, q, k, m, u, du, lse, dq, dk, sc, a.drop, 7, keep=keep,
                                   koff=koff)
    pairs = B * Lq * sum(lks)
    prev = lib().s2h_attn_config(1)
    vs = [int(v) for v in a.variants.split(",")]
    res = {v: [] for v in vs}
    try:
        for _ in range(a.rounds):
            for v in vs:
                lib().s2h_attn_config(v)
                res[v].append(timeit(bwd, a.iters))
    finally:
        lib().s2h_attn_config(prev)
    for v, ts in res.items():
        t = min(ts)
        # flops per (query, key): dQ kernel 2 (2 D + DV) + dK kernel 2 (2 D + DV)
        print(f"variant {v}: bwd {t:.3f} ms (min of {len(ts)}; all {', '.join(f'{x:.3f}' for x in ts)})  "
              f"{4 * (2 * 256 + 64) * pairs / t / 1e9:.0f} TF/s", flush=True)


if __name__ == "__main__":
    main()
