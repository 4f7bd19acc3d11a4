"""Which Python lines of the training step still launch stock PyTorch (at::native) kernels: one eager
step of the bench workload under a TorchDispatchMode; every aten op on CUDA tensors (views excluded)
is listed with the elements it produced and the innermost sam2_video frames that issued it.
    python tools/native_sites.py [--frames 8] [--top 40]"""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))

import argparse  # noqa: E402

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--top", type=int, default=60)
    ap.add_argument("--ops", default="", help="comma list of s2h_* entry points: report their call sites instead")
    a = ap.parse_args()
    from sam2_video.data.synthetic import make_clip, sam2_collate_fn
    from sam2_video.kernels import functional as FN
    from sam2_video.model.sam2model import SAM2Model
    from sam2_video.training.trainer import SAM2LightningModule, StepRunner

    dev = torch.device("cuda", 0)
    FN.set_seed(1234)
    ALL = ["image_encoder", "memory_attention", "memory_encoder", "mask_decoder", "prompt_encoder"]
    model = SAM2Model(None, "base_plus@512", trainable_modules=ALL, compute_dtype="bf16")
    loss_cfg = {"type": "multi_step", "gt_stride": 1, "multistep_logit_temperature": 1.0,
                "weight_dict": {"loss_mask": 20, "loss_dice": 1, "loss_iou": 1, "loss_class": 0},
                "supervise_all_iou": True, "iou_use_l1_loss": True, "pred_obj_scores": False,
                "focal_gamma_obj_score": 0.0, "focal_alpha_obj_score": -1.0}
    opt_cfg = {"type": "AdamW", "lr": 4e-6, "weight_decay": 0.01, "betas": [0.9, 0.999], "warmup_factor": 0.15}
    module = SAM2LightningModule(model, loss_cfg, opt_cfg, {"enabled": True, "num_cycles": 0.5})
    module.setup("fit", dev)
    runner = StepRunner(module, total_steps=4, distributed=False, graph=False)
    batches = [sam2_collate_fn([make_clip(i, a.frames, 512, 13, 13)]).to(dev) for i in range(3)]
    for b in batches[:2]:
        runner(b)
    torch.cuda.synchronize()
    import traceback
    from torch.utils._python_dispatch import TorchDispatchMode

    agg = collections.defaultdict(lambda: [0, 0])

    class Sites(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            out = func(*args, **(kwargs or {}))
            name = str(func.overloadpacket.__name__)
            ts = [t for t in list(args) + list((kwargs or {}).values()) if isinstance(t, torch.Tensor)]
            if any(t.is_cuda for t in ts) and name not in ("view", "as_strided", "empty", "empty_strided",
                                                           "_unsafe_view", "detach", "t", "transpose",
                                                           "permute", "unsqueeze", "squeeze", "expand",
                                                           "select", "slice", "reshape", "alias", "unbind",
                                                           "split", "split_with_sizes", "chunk", "narrow",
                                                           "is_same_size", "_local_scalar_dense"):
                fr = [f for f in traceback.extract_stack() if "sam2_video" in f.filename][-3:]
                where = " <- ".join(f"{f.filename.split('sam2_video/')[-1]}:{f.lineno}" for f in reversed(fr))
                o = out if isinstance(out, torch.Tensor) else (out[0] if isinstance(out, (list, tuple)) and out
                                                                and isinstance(out[0], torch.Tensor) else None)
                agg[(name, where)][0] += 1
                agg[(name, where)][1] += o.numel() if o is not None else 0
            return out

    if a.ops:
        from sam2_video.kernels import ops as _ops
        want = set(a.ops.split(","))
        real = _ops.call
        calls = collections.Counter()

        def spy(name, *args):
            if name in want:
                fr = [f for f in traceback.extract_stack() if "sam2_video" in f.filename][-4:-1]
                where = " <- ".join(f"{f.filename.split('sam2_video/')[-1]}:{f.lineno}" for f in reversed(fr))
                # inside the frame tape's backward: which op's input gradient is being accumulated
                f0 = sys._getframe(1)
                while f0 is not None and not (f0.f_code.co_name == "backward" and "frametape" in f0.f_code.co_filename):
                    f0 = f0.f_back
                if f0 is not None and "op" in f0.f_locals:
                    op = f0.f_locals["op"]
                    where += f"  [tape op {getattr(op, 'kind', '?')} #{getattr(op, 'idx', '?')}, n={args[1] if len(args) > 1 else '?'}]"
                calls[(name, where)] += 1
            return real(name, *args)

        _ops.call = spy
        runner(batches[2])
        torch.cuda.synchronize()
        _ops.call = real
        for (name, where), n in calls.most_common(a.top):
            print(f"n={n:4d}  {name:20s} {where}")
        return
    with Sites():
        runner(batches[2])
    torch.cuda.synchronize()
    print(f"aten ops with CUDA tensors in one eager step: {sum(v[0] for v in agg.values())}")
    for (name, where), (n, el) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{el / 1e6:9.2f} M elems  n={n:4d}  {name:24s} {where}")


if __name__ == "__main__":
    main()
