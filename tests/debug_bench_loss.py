"""Debug helper (not a test): per-step losses of the bench workload, graphed, batches resident
up front like bench.py; after each step, checks the graph's static inputs against the batch."""
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
size, S, T, O, n = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
FN.set_seed(1234)
model = SAM2Model(None, f"{size}@{S}", trainable_modules=ALL, compute_dtype="bf16")
opt = {"type": "AdamW", "lr": 4e-6, "weight_decay": 0.01, "betas": [0.9, 0.999], "warmup_factor": 0.15}
module = SAM2LightningModule(model, LOSS, opt, {"enabled": True, "num_cycles": 0.5})
module.setup("fit", "cuda")
run = StepRunner(module, total_steps=n, graph=True)
batches = [sam2_collate_fn([make_clip(i, T, S, O, O)]).to("cuda") for i in range(n)]
torch.cuda.synchronize()
for i in range(n):
    loss = float(run(batches[i]).detach())
    ent = next(iter(run._graphs.values()))
    st = ent["batch"]
    ok_img = torch.equal(st.img_batch, batches[i].img_batch)
    ok_m = torch.equal(st.masks, batches[i].masks)
    plan = model.host_prompt_plan(batches[i])
    dev = st.prompt_plan["dev"]
    ok_p = all(torch.equal(d.cpu(), h) for d, h in zip(dev, plan["host"]))
    # replay again on the same inputs (no optimizer step): same loss?
    ent["graph"].replay()
    again = float(ent["loss"].detach())
    print(f"step {i} loss {loss:.5f} replay-again {again:.5f} img {ok_img} masks {ok_m} prompts {ok_p}", flush=True)
