"""Event timing of the V-fold memory cross-attention backward as the bench step runs it: one
frame-table launch over 7 frames (memory banks of 1..7 frames x 1028 keys), 13 objects x 1024
queries, head dim 256, dropout 0.1 with the forward's keep bitmap.  One line per attention
variant (s2h_attn_config values, default "1"), the variants interleaved over rounds:
    python tools/vfold_bwd_bench.py [--variants 1,33] [--iters 10] [--rounds 2]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))

import torch  # noqa: E402

from sam2_video.kernels import ops  # noqa: E402
from sam2_video.kernels._lib import lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="1")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--drop", type=float, default=0.1)
    a = ap.parse_args()
    dev, bf = "cuda", torch.bfloat16
    B, Lq, scale, seed = 13, 1024, 256 ** -0.5, 7
    lks = [1028 * m for m in range(1, 8)]
    g = torch.Generator(device="cpu").manual_seed(0)
    idx0, koff, krow, acc_e, acc_w, acc_k = [], [], [], 0, 0, 0
    qs, ks, ms, us, lses, keeps = [], [], [], [], [], []
    for lk in lks:
        q = (torch.randn(B, Lq, 1, 256, generator=g) * 0.5).to(dev, bf)
        k = (torch.randn(B, lk, 1, 256, generator=g) * 0.5).to(dev, bf)
        m = torch.randn(B, lk, 1, 64, generator=g).to(dev, bf)
        u = torch.empty(B, Lq, 1, 72, device=dev, dtype=bf)
        lse = torch.empty(B, 1, Lq, device=dev)
        keep = torch.zeros(ops.keep_words(B, 1, Lq, lk), device=dev, dtype=torch.int32)
        ops.attn_fwd_vfold(q, k, m, u, lse, scale, a.drop, seed, idx0=acc_e, keep=keep if a.drop > 0 else None)
        idx0.append(acc_e)
        koff.append(acc_w)
        krow.append(acc_k)
        acc_e += B * Lq * lk
        acc_w += keep.numel()
        acc_k += B * lk
        qs.append(q), ks.append(k.reshape(-1, 1, 256)), ms.append(m.reshape(-1, 1, 64))
        us.append(u), lses.append(lse), keeps.append(keep)
    q_all, k_all, m_all, u_all = torch.cat(qs), torch.cat(ks), torch.cat(ms), torch.cat(us)
    lse_all, keep_all = torch.cat(lses), torch.cat(keeps)
    du = (torch.randn(u_all.shape, generator=g) * 0.1).to(dev, bf)
    dq, dk = torch.empty_like(q_all), torch.empty_like(k_all)

    def run():
        ops.flash_bwd_frames_vfold(len(lks), B, lks, krow, idx0, q_all, k_all, m_all, u_all, du, lse_all, dq, dk,
                                   scale, a.drop, seed, keep=keep_all if a.drop > 0 else None,
                                   koff=koff if a.drop > 0 else None)

    variants = [int(v) for v in a.variants.split(",")]
    prev = lib().s2h_attn_config(1)
    res = {v: [] for v in variants}
    try:
        for _ in range(a.rounds):
            for v in variants:
                lib().s2h_attn_config(v)
                for _ in range(2):
                    run()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(a.iters):
                    run()
                e.record()
                torch.cuda.synchronize()
                res[v].append(s.elapsed_time(e) / a.iters)
    finally:
        lib().s2h_attn_config(prev)
    for v in variants:
        print(f"variant {v}: V-fold backward (dQ + dK) {' / '.join(f'{t:.3f}' for t in res[v])} ms", flush=True)


if __name__ == "__main__":
    main()
