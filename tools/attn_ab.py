"""A/B timing of the memory-attention flash kernels as the training step runs them: forward
with dropout 0.1 writing the keep bitmap (cross-attention shapes, 13 objects x 1024 queries x
1028 n keys, and self-attention 1024 keys), then the frame-table backward over 7 frames reading
it.  Run once per build: S2H_LIB_PATH=<lib> python tools/attn_ab.py [--iters 20]"""
import argparse
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))

import torch  # noqa: E402

from sam2_video.kernels import ops  # noqa: E402


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
    ap.add_argument("--drop", type=float, default=0.1)
    ap.add_argument("--variants", action="store_true", help="also time the backward with s2h_attn_config(3)")
    ap.add_argument("--targets", default="", help="comma list of flash-forward key-split targets (workgroups) to sweep")
    a = ap.parse_args()
    if a.targets:
        from sam2_video.kernels._lib import lib
        for t in a.targets.split(","):
            lib().s2h_attn_config(1 | (int(t) << 8))
            print(f"key-split target {t}:", end=" ")
            run(a)
        lib().s2h_attn_config(1)
        return
    run(a)


def run(a):
    torch.manual_seed(0)
    B, Lq, H, D = 13, 1024, 1, 256
    sc = 1 / math.sqrt(D)
    out = [os.path.basename(os.environ.get("S2H_LIB_PATH", "default"))]
    for name, lks in (("cross", [1028 * n for n in range(1, 8)]), ("self", [1024] * 7)):
        F = len(lks)
        q = (torch.randn(F * B, Lq, H, D, device="cuda") * 0.5).to(torch.bfloat16)
        rows = sum(B * lk for lk in lks)
        k = (torch.randn(rows, H, D, device="cuda") * 0.5).to(torch.bfloat16)
        v = torch.randn(rows, H, D, device="cuda").to(torch.bfloat16)
        do = torch.randn_like(q)
        o = torch.empty_like(q)
        lse = torch.empty(F * B, H, Lq, device="cuda")
        nw = [ops.keep_words(B, H, Lq, lk) for lk in lks]
        koff = [sum(nw[:f]) for f in range(F)]
        keep = torch.empty(sum(nw), device="cuda", dtype=torch.int32)
        krow, idx0, r, n = [], [], 0, 0
        for lk in lks:
            krow.append(r)
            idx0.append(n)
            r += B * lk
            n += B * H * Lq * lk

        def fwd():
            for f, lk in enumerate(lks):
                sl = slice(f * B, (f + 1) * B)
                r0 = krow[f]
                ops.attn_fwd(q[sl], k[r0:r0 + B * lk].view(B, lk, H, D), v[r0:r0 + B * lk].view(B, lk, H, D), o[sl],
                             lse[sl], sc, a.drop, 7, idx0=idx0[f], keep=keep[koff[f]:koff[f] + nw[f]])
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)

        def bwd():
            ops.flash_bwd_frames(F, B, lks, krow, idx0, q, k, v, o, do, lse, dq, dk, dv, sc, a.drop, 7, keep=keep,
                                 koff=koff)
        tf, tb = timeit(fwd, a.iters), timeit(bwd, a.iters)
        fl = 4.0 * B * H * Lq * sum(lks) * D
        out.append(f"{name}: fwd {tf:.3f} ms ({fl / tf / 1e9:.0f} TF/s)  bwd {tb:.3f} ms ({2.5 * fl / tb / 1e9:.0f} TF/s)")
        if a.variants:  # the same backward with the one-wave-per-SIMD dK / dV kernel (s2h_attn_config 3)
            from sam2_video.kernels._lib import lib
            prev = lib().s2h_attn_config(3)
            try:
                tb3 = timeit(bwd, a.iters)
            finally:
                lib().s2h_attn_config(prev)
            out.append(f"(bwd with the 32x32 dK/dV kernel {tb3:.3f} ms)")
    print("  ".join(out), flush=True)


if __name__ == "__main__":
    main()
