"""Eager-vs-eager and eager-vs-graph-replay comparison of one training step (diagnostic).

For a config (model, image size, frames, objects, dtype) runs the SAME clip through
  (a) an eager StepRunner step on a fresh module,
  (b) a second eager step on another fresh module (determinism of the eager step),
  (c) a graph StepRunner step (warm-up + capture + one replay) on a fresh module,
and prints, per frame, the max |difference| of the category-level low-res logits between (a) and
(b) / (a) and (c), plus the backbone outputs and the loss, so the first frame / stage where a
replay departs from eager is visible.

  python tools/replay_diff.py --dtype fp8 --frames 16 --size 512
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402


def run(args, graph):
    from test_configs_gpu import _clips, _module
    from sam2_video.training.trainer import StepRunner
    mod = _module(args.model, args.size, dtype=args.dtype, lr=args.lr, dropout=args.dropout)
    clip = _clips([args.clip], args.frames, args.size, args.objects, args.objects)[0]
    run = StepRunner(mod, total_steps=1, graph=graph)
    loss = float(run(clip).detach())
    torch.cuda.synchronize()
    outs = [fr["pred_masks"].detach().float().clone() for fr in mod.last_outputs]
    bb = [t.detach().float().clone() for t in (mod.model.last_backbone_outputs or [])]
    grad = mod.model.arena.grad_region().detach().clone()
    del run, mod
    torch.cuda.empty_cache()
    return loss, outs, bb, grad


def compare(name, a, b):
    la, oa, ba, ga = a
    lb, ob, bbb, gb = b
    print(f"== {name}: loss {la:.7f} vs {lb:.7f} (rel {abs(la - lb) / max(1e-12, abs(la)):.3e})")
    for i, (x, y) in enumerate(zip(ba, bbb)):
        print(f"   backbone[{i}] max|d| {(x - y).abs().max().item():.3e}  bitwise {torch.equal(x, y)}")
    first = None
    for t, (x, y) in enumerate(zip(oa, ob)):
        d = (x - y).abs().max().item()
        if d > 0 and first is None:
            first = t
        print(f"   frame {t:2d} max|dlogit| {d:.3e}  mask flips {int(((x > 0) != (y > 0)).sum())}")
    dg = (ga - gb).abs().max().item()
    print(f"   first differing frame: {first}; grad arena max|d| {dg:.3e} (max |g| {ga.abs().max().item():.3e})")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="base_plus")
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--objects", type=int, default=13)
    ap.add_argument("--dtype", default="fp8")
    ap.add_argument("--clip", type=int, default=70)
    ap.add_argument("--lr", type=float, default=1e-5)
    ap.add_argument("--dropout", type=float, default=None)
    ap.add_argument("--skip-eager2", action="store_true")
    args = ap.parse_args()
    print(vars(args), flush=True)
    e1 = run(args, False)
    if not args.skip_eager2:
        e2 = run(args, False)
        compare("eager vs eager", e1, e2)
    g = run(args, True)
    compare("eager vs graph replay", e1, g)


if __name__ == "__main__":
    main()
