"""Which op of the tracking loop makes two identical forwards differ? (diagnostic)

Runs the training-mode forward (frame tapes recording) of one clip several times with the same
weights, host seeds and device RNG offset, and compares every value the frame tapes stored --
per tape, frame and op output, in execution order -- between the runs.  Between runs the caching
allocator's free memory is overwritten (NaN, then random bits), so an op that reads memory it
did not write shows up as a difference.

  python tools/tape_diff.py --dtype bf16 --frames 8 --size 512
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

TRACKERS = []


def _hook():
    from sam2_video.model import tracking
    init = tracking.FrameTracker.__init__

    def wrapped(self, *a, **k):
        init(self, *a, **k)
        TRACKERS.append(self)
    tracking.FrameTracker.__init__ = wrapped


def snapshot(tr):
    """[(tape name, frame, op index, op kind, value id, tensor)] in execution order"""
    out = []
    tapes = ([tr.ma] if tr.ma is not None else []) + [tp for tp, _ in tr.decs]
    for tp in tapes:
        prod = {}
        for i, op in enumerate(tp.ops):
            for v in op.outs:
                if v is not None and v not in prod:
                    prod[v] = (i, op.kind)
        vids = list(tp.stores)
        for f in range(tp.F):
            for v in vids:
                st = tp.stores[v]
                i, kind = prod.get(v, (-1, str(v[0]) if isinstance(v, tuple) else "?"))
                out.append((tp.name, f, i, kind, v, st.frame(f).detach().float().cpu().clone()))
    return out


def garble(mode, gb):
    torch.cuda.synchronize()
    n = int(gb * (1 << 30)) // 4
    x = torch.empty(n, dtype=torch.float32, device="cuda")
    if mode == "nan":
        x.fill_(float("nan"))
    else:
        x.random_()
    torch.cuda.synchronize()
    del x


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="base_plus")
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--objects", type=int, default=13)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--dropout", type=float, default=0.1)
    ap.add_argument("--clip", type=int, default=70)
    ap.add_argument("--garble-gb", type=float, default=24.0)
    ap.add_argument("--show", type=int, default=25)
    args = ap.parse_args()
    print(vars(args), flush=True)
    _hook()
    from step_harness import ALL, build_model
    from test_configs_gpu import _clips
    from sam2_video.kernels import functional as FN
    from sam2_video.kernels.ops import rng_offset
    m = build_model(args.model, args.size, ALL, dtype=args.dtype, dropout=args.dropout)
    clip = _clips([args.clip], args.frames, args.size, args.objects, args.objects)[0]
    rng = rng_offset(m.arena.device)
    snaps, outs = [], []
    for r, mode in enumerate(["none", "nan", "rand"]):
        if mode != "none":
            garble(mode, args.garble_gb)
        FN.set_seed(777)
        rng.fill_(1)
        TRACKERS.clear()
        res, _ = m(clip)
        torch.cuda.synchronize()
        outs.append([fr["pred_masks"].detach().float().cpu() for fr in res])
        snaps.append(snapshot(TRACKERS[-1]))
        del res
        print(f"run {r} ({mode}): {len(snaps[-1])} tape values", flush=True)
    for r in (1, 2):
        print(f"== run 0 vs run {r}")
        nd, nan = 0, 0
        for a, b in zip(snaps[0], snaps[r]):
            assert a[:5] == b[:5]
            x, y = a[5], b[5]
            same = torch.equal(x, y) or (torch.isnan(x) == torch.isnan(y)).all() and torch.equal(
                torch.nan_to_num(x), torch.nan_to_num(y))
            if not same:
                if nd < args.show:
                    d = (x - y).abs()
                    print(f"   {a[0]} frame {a[1]} op {a[2]} {a[3]} {a[4]}: max|d| {torch.nan_to_num(d, 1e30).max().item():.3e}"
                          f" ndiff {int((x != y).sum())}/{x.numel()} nan {int(torch.isnan(y).sum())}")
                    if nd < 3:  # where: (row, col) of a [rows, last dim] view, the two values
                        x2, y2 = x.reshape(-1, x.shape[-1]), y.reshape(-1, y.shape[-1])
                        idx = (x2 != y2).nonzero()[:40].tolist()
                        print("      at", [(r, c, round(x2[r, c].item(), 4), round(y2[r, c].item(), 4)) for r, c in idx])
                nd += 1
            if torch.isnan(b[5]).any():
                nan += 1
        print(f"   {nd} differing tape values, {nan} with NaN")
        for t, (x, y) in enumerate(zip(outs[0], outs[r])):
            print(f"   frame {t} logits max|d| {(x - y).abs().max().item():.3e}")


if __name__ == "__main__":
    main()
