"""Which host-side ops launch the torch (non-libsam2hip) kernels of a training step?

Runs warmup steps of the bench workload, then one step under torch.profiler and prints
(a) the aten ops by device time and (b) the Python call sites of the copy / fill / add /
cat launches.  GPU only.

  python tools/torch_prof.py [--frames 8] [--rows 40]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--image-size", type=int, default=512)
    ap.add_argument("--objects", type=int, default=13)
    ap.add_argument("--rows", type=int, default=40)
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
    runner = StepRunner(module, 10, graph=False)  # eager: the profiler sees each launch and its call site
    batch = sam2_collate_fn([make_clip(0, a.frames, a.image_size, a.objects, a.objects)]).to("cuda")
    for _ in range(2):
        runner(batch)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True, record_shapes=True) as prof:
        runner(batch)
        torch.cuda.synchronize()
    ka = prof.key_averages()
    print(ka.table(sort_by="self_device_time_total", row_limit=a.rows, max_name_column_width=60))
    # call sites of the torch copies / fills / adds / cats
    want = ("aten::copy_", "aten::fill_", "aten::add_", "aten::add", "aten::cat", "aten::zero_", "aten::clone",
            "aten::contiguous", "aten::index", "aten::mul", "aten::stack")
    # forward ops by autograd sequence number (a backward node's ops carry the forward op's number)
    fwd_by_seq = {}
    for ev in prof.events():
        sq = getattr(ev, "sequence_nr", -1)
        if sq is not None and sq >= 0 and ev.stack and not ev.name.startswith("autograd::"):
            fwd_by_seq.setdefault(sq, ev)
    sites = {}
    for ev in prof.events():
        if ev.name not in want:
            continue
        dev = getattr(ev, "self_device_time_total", 0) or 0
        if dev <= 0:
            continue
        stack = [s for s in (ev.stack or []) if "sam2_video" in s or "tests" in s or "bench" in s]
        if stack:
            where = " <- ".join(stack[:3])
        else:  # backward-engine ops have no Python frame: name the enclosing ops instead
            chain, p, fwd = [], ev.cpu_parent, None
            while p is not None and len(chain) < 4:
                chain.append(p.name)
                sq = getattr(p, "sequence_nr", -1)
                if fwd is None and sq is not None and sq >= 0 and sq in fwd_by_seq:
                    fwd = fwd_by_seq[sq]
                p = p.cpu_parent
            where = "parents: " + " < ".join(chain[:2]) if chain else "(no python frame)"
            if fwd is not None:
                fst = [s for s in fwd.stack if "sam2_video" in s or "tests" in s]
                where += " | fwd " + fwd.name + " @ " + " <- ".join(fst[:3])
        key = (ev.name, where)
        v = sites.setdefault(key, [0, 0.0])
        v[0] += 1
        v[1] += dev
    print("\n# device time by call site (us)")
    for (name, st), (n, t) in sorted(sites.items(), key=lambda kv: -kv[1][1])[:60]:
        print(f"{t:10.1f} us n={n:4d} {name:18s} {st}")


if __name__ == "__main__":
    main()
