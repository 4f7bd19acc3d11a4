"""Python call sites of the stock-torch device ops (copies, fills, cats, adds) of one eager training
step, counted per site.  torch.profiler's with_stack gives no frames on this image, so this records
them itself: a TorchDispatchMode sees every aten op issued in this thread, and the backward runs in
this thread too (autograd multithreading off).  GPU only.

  python tools/copy_sites.py [--frames 8] [--rows 50]
"""
import argparse
import collections
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

WANT = {"copy_", "fill_", "zero_", "cat", "stack", "add", "add_", "clone", "_to_copy", "repeat_interleave",
        "index", "index_put_", "mul", "mul_", "sub", "div", "where", "masked_fill_", "sum",
        "_copy_from", "select_backward", "slice_backward", "copy"}


class Sites(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.count = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = func.overloadpacket.__name__
        if name in WANT:
            devs = [a for a in list(args) + list((kwargs or {}).values()) if isinstance(a, torch.Tensor)]
            if any(t.is_cuda for t in devs) or (isinstance(out, torch.Tensor) and out.is_cuda):
                fr = [f for f in traceback.extract_stack()[:-1] if "sam2_video" in f.filename]
                site = " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}:{f.name}" for f in reversed(fr[-3:]))
                self.count[(name, site or "(no sam2_video frame)")] += 1
        return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--image-size", type=int, default=512)
    ap.add_argument("--objects", type=int, default=13)
    ap.add_argument("--rows", type=int, default=60)
    ap.add_argument("--ops", nargs="*", default=[], help="kernels.ops functions whose call sites to count")
    a = ap.parse_args()
    from sam2_video.data.synthetic import make_clip, sam2_collate_fn
    from sam2_video.model.sam2model import SAM2Model
    from sam2_video.training.trainer import SAM2LightningModule, StepRunner

    ALL = ["image_encoder", "memory_attention", "memory_encoder", "mask_decoder", "prompt_encoder"]
    model = SAM2Model(None, f"base_plus@{a.image_size}", trainable_modules=ALL, compute_dtype="bf16")
    loss_cfg = {"type": "multi_step", "weight_dict": {"loss_mask": 20, "loss_dice": 1, "loss_iou": 1, "loss_class": 0},
                "supervise_all_iou": True, "iou_use_l1_loss": True}
    module = SAM2LightningModule(model, loss_cfg, {"type": "AdamW", "lr": 4e-6}, {"enabled": False})
    module.setup("fit", "cuda")
    runner = StepRunner(module, 10, graph=False)
    batch = sam2_collate_fn([make_clip(0, a.frames, a.image_size, a.objects, a.objects)]).to("cuda")
    for _ in range(2):
        runner(batch)
    torch.cuda.synchronize()
    torch.autograd.set_multithreading_enabled(False)
    # the library's own element-wise launches named on the command line (--ops add add_bcast ...):
    # wrapped to count their call sites too
    from sam2_video.kernels import ops as _ops
    lib_count = collections.Counter()

    def wrap(name):
        fn = getattr(_ops, name)

        def w(*args, **kw):
            fr = [f for f in traceback.extract_stack()[:-1] if "sam2_video" in f.filename and "ops.py" not in f.filename]
            lib_count[(name, " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}:{f.name}"
                                         for f in reversed(fr[-3:])))] += 1
            return fn(*args, **kw)
        setattr(_ops, name, w)
    for name in a.ops:
        wrap(name)
    mode = Sites()
    with mode:
        runner(batch)
    torch.cuda.synchronize()
    if lib_count:
        print(f"# library launches by call site ({sum(lib_count.values())})")
        for (name, site), n in lib_count.most_common(a.rows):
            print(f"{n:5d} {name:18s} {site}")
    total = sum(mode.count.values())
    print(f"# {total} stock-op calls on CUDA tensors in one step (not all launch a kernel: views / no-ops too)")
    for (name, site), n in mode.count.most_common(a.rows):
        print(f"{n:5d} {name:18s} {site}")


if __name__ == "__main__":
    main()
