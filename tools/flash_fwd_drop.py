"""Cost of the in-softmax dropout in the flash forward on the memory-attention shapes: the V-fold
cross-attention (13 objects x 1024 queries x 1028 n keys, n = 1..7, as the 7 memory frames of a
step) and the self-attention (1024 keys), each with p = 0, p = 0.1 hash-only and p = 0.1 writing
the keep bitmap (the training step's form).  GPU only.
  python tools/flash_fwd_drop.py [--iters 10] [--rounds 3]   (S2H_LIB_PATH selects the build)"""
import argparse
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
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    torch.manual_seed(0)
    B, Lq = 13, 1024
    lks = [1028 * n for n in range(1, 8)]
    bf = torch.bfloat16
    sc = 256 ** -0.5
    q = (torch.randn(B, Lq, 1, 256, device="cuda") * 0.5).to(bf)
    k = (torch.randn(B, lks[-1], 1, 256, device="cuda") * 0.5).to(bf)
    m = torch.randn(B, lks[-1], 1, 64, device="cuda").to(bf)
    v = torch.randn(B, 1024, 1, 256, device="cuda").to(bf)
    u = torch.empty(B, Lq, 1, 72, device="cuda", dtype=bf)
    o = torch.empty(B, Lq, 1, 256, device="cuda", dtype=bf)
    lse = torch.empty(B, 1, Lq, device="cuda")
    keep = torch.zeros(ops.keep_words(B, 1, Lq, lks[-1]), device="cuda", dtype=torch.int32)

    def cross(p, kp):
        def f():
            for lk in lks:
                ops.attn_fwd_vfold(q, k[:, :lk], m[:, :lk], u, lse, sc, p, 7, idx0=0,
                                   keep=keep[:ops.keep_words(B, 1, Lq, lk)] if kp else None)
        return f

    def self_(p, kp):
        def f():
            for _ in range(7):
                ops.attn_fwd(q, k[:, :1024], v, o, lse, sc, p, 7, keep=keep[:ops.keep_words(B, 1, Lq, 1024)]
                                    if kp else None)
        return f
    flops_x = sum(2 * (256 + 64) * B * Lq * lk for lk in lks)
    flops_s = 7 * 2 * 512 * B * Lq * 1024
    for name, mk, fl in (("cross V-fold x7", cross, flops_x), ("self x7", self_, flops_s)):
        for p, kp, tag in ((0.0, False, "p=0"), (0.1, False, "p=0.1 hash"), (0.1, True, "p=0.1 bitmap")):
            ts = [timeit(mk(p, kp), a.iters) for _ in range(a.rounds)]
            t = min(ts)
            print(f"{name:16s} {tag:13s} {t * 1e3 / 7:7.1f} us/launch  {fl / (t * 1e-3) / 1e12:6.0f} TF/s", flush=True)


if __name__ == "__main__":
    main()
