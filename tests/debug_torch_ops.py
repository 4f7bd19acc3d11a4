"""Debug helper (not a test): which torch-side ops (adds, copies, fills) run in one eager bench
step, attributed to the autograd node / Python frame that issued them."""
import collections
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "sam2-video-training_amd"))
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from sam2_video.data.synthetic import make_clip, sam2_collate_fn  # noqa: E402
from sam2_video.model.sam2model import SAM2Model  # noqa: E402
from sam2_video.training.trainer import SAM2LightningModule, StepRunner  # noqa: E402

ALL = ["image_encoder", "memory_attention", "memory_encoder", "mask_decoder", "prompt_encoder"]
LOSS = {"type": "multi_step", "gt_stride": 1, "multistep_logit_temperature": 1.0,
        "weight_dict": {"loss_mask": 20, "loss_dice": 1, "loss_iou": 1, "loss_class": 0},
        "supervise_all_iou": True, "iou_use_l1_loss": True, "pred_obj_scores": False}
model = SAM2Model(None, "base_plus@512", trainable_modules=ALL, compute_dtype="bf16")
opt = {"type": "AdamW", "lr": 4e-6, "weight_decay": 0.01, "betas": [0.9, 0.999], "warmup_factor": 0.15}
module = SAM2LightningModule(model, LOSS, opt, {"enabled": False})
module.setup("fit", "cuda")
run = StepRunner(module, total_steps=4, graph=False)
b = sam2_collate_fn([make_clip(0, 8, 512, 13, 13)]).to("cuda")
run(b)
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=True) as prof:
    run(b)
    torch.cuda.synchronize()
agg = collections.Counter()
for ev in prof.events():
    if ev.name in ("aten::add_", "aten::add", "aten::copy_", "aten::fill_", "aten::zero_", "aten::zeros",
                   "aten::cat", "aten::clone", "aten::contiguous", "aten::sum", "aten::mul"):
        st = [f for f in (ev.stack or []) if "sam2_video" in f or "autograd" in f][:3]
        agg[(ev.name, str(ev.input_shapes)[:60], " | ".join(s.split("/")[-1] for s in st))] += 1
for (name, shp, st), n in agg.most_common(45):
    print(f"{n:5d} {name:14s} {shp:60s} {st}")
