"""Shared helpers: run one training step of the HIP build on the GPU and compare it
with golden fixtures from the reference / with the CPU oracle (tests only)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
ALL = ["image_encoder", "memory_attention", "memory_encoder", "mask_decoder", "prompt_encoder"]
CASES = {
    "tiny256_point_all": ("tiny", "point", ALL),
    "tiny256_point_mem": ("tiny", "point", ["memory_attention", "memory_encoder"]),
    "tiny256_box_all": ("tiny", "box", ALL),
    "bplus128_point_all": ("base_plus", "point", ALL),
    "bplus128_point_all_t8": ("base_plus", "point", ALL),
    "tiny256_point_all_multi": ("tiny", "point", ALL),
    "tiny256_mask_all": ("tiny", "mask", ALL),
    "bplus256_point_all": ("base_plus", "point", ALL),
    # Hiera-L trunk (BASELINE config 4's model): stages [2, 6, 36, 4], head dim 72
    "large128_point_all": ("large", "point", ALL),
}
# reference steps under CPU bf16 autocast (oracle/gen_golden.py), with their fp32 twin
BF16_CASES = {"bplus256_point_all_bf16": "bplus256_point_all"}


def load_golden(name):
    return torch.load(os.path.join(GOLD, name + ".pt"), weights_only=True)


def build_model(size, image_size, trainable, prompt="point", dtype="fp32", seed=0, dropout=0.0):
    from sam2_video.model.sam2model import SAM2Model
    m = SAM2Model(None, f"{size}@{image_size}", trainable_modules=trainable, prompt_type=prompt, compute_dtype=dtype,
                  init_seed=seed)
    m.load("cuda")
    m.train()
    m.set_dropout(dropout)
    return m


def run_step(model, batch, criterion=None):
    """forward (keeping per-object outputs) + loss + backward; returns (stages, merged, losses)"""
    from sam2_video.model.losses import MultiStepMultiMasksAndIous
    from sam2_video.utils.masks import merge_object_results_to_category
    if criterion is None:
        criterion = MultiStepMultiMasksAndIous({"loss_mask": 20, "loss_dice": 1, "loss_iou": 1, "loss_class": 0},
                                               supervise_all_iou=True, iou_use_l1_loss=True)
    model.arena.zero_grad()
    bo = model.forward_image(batch.flat_img_batch)
    bo = model.prepare_prompt_inputs(bo, batch)
    stages = model.forward_tracking(bo, batch)
    merged = merge_object_results_to_category(stages, bo["obj_to_cat"], bo["num_categories"])
    losses = criterion(merged, batch.masks)
    losses["total_loss"].backward()
    torch.cuda.synchronize()
    return stages, merged, losses, bo


def golden_batch(g):
    from sam2_video.data.synthetic import synthetic_batch
    T, S = int(g["meta/T"]), int(g["meta/image_size"])
    n_cat = g["in/masks_count"].shape[1]
    n_obj = int((g["in/masks_count"][0] > 0).sum())
    parts = g["meta/parts"].tolist() if "meta/parts" in g else None
    return synthetic_batch(int(g["meta/clip_idx"]), T, S, n_cat, n_obj, parts)


def grads_by_name(model):
    out = {}
    for n, p in model.named_parameters():
        gv = getattr(p, "_s2h_grad", None)
        if gv is not None:
            out[n] = gv.detach().float().cpu()
    return out


def mask_iou(a, b):
    a, b = a > 0, b > 0
    inter = (a & b).sum().item()
    uni = (a | b).sum().item()
    return inter / max(uni, 1)
