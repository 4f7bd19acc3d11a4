"""Debug helper (not a test): replay the captured bench step many times on one clip with
lr = 0 and no host syncs; every replay must give the same loss."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "sam2-video-training_amd"))
import torch  # noqa: E402

from sam2_video.data.synthetic import make_clip, sam2_collate_fn  # noqa: E402
from sam2_video.kernels import functional as FN  # noqa: E402
from sam2_video.model.sam2model import SAM2Model  # noqa: E402
from sam2_video.training.trainer import SAM2LightningModule, StepRunner  # noqa: E402

ALL = ["image_encoder", "memory_attention", "memory_encoder", "mask_decoder", "prompt_encoder"]
LOSS = {"type": "multi_step", "gt_stride": 1, "multistep_logit_temperature": 1.0,
        "weight_dict": {"loss_mask": 20, "loss_dice": 1, "loss_iou": 1, "loss_class": 0},
        "supervise_all_iou": True, "iou_use_l1_loss": True, "pred_obj_scores": False}
mode = sys.argv[1]
drop, lr = float(sys.argv[2]), float(sys.argv[3])
FN.set_seed(1234)
model = SAM2Model(None, "base_plus@512", trainable_modules=ALL, compute_dtype="bf16")
model.set_dropout(drop)
opt = {"type": "AdamW", "lr": lr, "weight_decay": 0.01, "betas": [0.9, 0.999], "warmup_factor": 0.0}
module = SAM2LightningModule(model, LOSS, opt, {"enabled": False})
module.setup("fit", "cuda")
run = StepRunner(module, total_steps=20, graph=(mode == "graph"))
batches = [sam2_collate_fn([make_clip(i % 2, 8, 512, 13, 13)]).to("cuda") for i in range(20)]
torch.cuda.synchronize()
losses = []
for i in range(20):
    losses.append(run(batches[i]).detach().clone())
    if mode == "graph-sync":
        torch.cuda.synchronize()
print(mode, drop, lr, [round(float(x), 5) for x in losses], flush=True)
