"""TEST INFRASTRUCTURE ONLY -- generates tests/golden/*.pt from the REFERENCE
itself (imported through oracle/ref_harness.py; this container only).

Each fixture = one full reference training step (SAM2Model.forward ->
MultiStepMultiMasksAndIous -> backward, restating SAM2LightningModule.training_step
trainer.py:256-289 without Lightning) on a deterministic synthetic clip with
deterministic synthetic weights, fp32, dropout disabled (parity mode).

Stored (all plain tensors, loadable with torch.load(weights_only=True)):
  inputs checksums, frame-0 point prompts, per-object low-res mask logits per
  frame, per-frame merged outputs (low-res masks, IoU preds, object scores,
  high-res sub-sampled logits + checksums), loss terms, per-parameter gradient
  norms / sums (full gradients for small tensors), the names of trainable
  parameters whose .grad stays None, and intermediate backbone features.

Usage:  python oracle/gen_golden.py [name ...]
"""
from __future__ import annotations

import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import ref_harness as H  # noqa: E402

OUT = os.path.join(os.path.dirname(HERE), "tests", "golden")

ALL = ["image_encoder", "memory_attention", "memory_encoder", "mask_decoder", "prompt_encoder"]
CASES = {
    # config 1 shape: Hiera-T, 256^2, 4 frames, 13 categories / 4 objects
    "tiny256_point_all": dict(size="tiny", image_size=256, T=4, n_cat=13, n_obj=4, prompt="point", trainable=ALL),
    "tiny256_point_mem": dict(size="tiny", image_size=256, T=4, n_cat=13, n_obj=4, prompt="point",
                              trainable=["memory_attention", "memory_encoder"]),
    "tiny256_box_all": dict(size="tiny", image_size=256, T=3, n_cat=5, n_obj=3, prompt="box", trainable=ALL),
    # Hiera-B+ structure (heads 2..16, head_dim 56, q-pool, global blocks 12/16/20) at a small resolution
    "bplus128_point_all": dict(size="base_plus", image_size=128, T=3, n_cat=4, n_obj=2, prompt="point",
                               trainable=ALL),
    # 8 frames: the full memory bank (cond frame + 6 previous frames = all 7 maskmem_tpos_enc slots),
    # object pointers from 8 frames and the non-cond bank prune (sam2model.py:365-377)
    "bplus128_point_all_t8": dict(size="base_plus", image_size=128, T=8, n_cat=4, n_obj=3, prompt="point",
                                  trainable=ALL),
    # categories split into 2 and 3 connected components: the max / sigmoid-mass weighted merge
    # over several objects (masks.py:53-213) and its gradient
    "tiny256_point_all_multi": dict(size="tiny", image_size=256, T=4, n_cat=5, n_obj=3, parts=(2, 3),
                                    prompt="point", trainable=ALL),
    # memory-attention Lq = 256 (flash-attention size) in fp32 and under CPU bf16 autocast: the
    # reference's own bf16 drift at the size where the bf16 kernels of the bench path run
    # mask prompts (sam2model.py:215-217): frame 0 bypasses the SAM heads (_use_mask_as_output)
    "tiny256_mask_all": dict(size="tiny", image_size=256, T=4, n_cat=5, n_obj=3, parts=(2,), prompt="mask",
                             trainable=ALL),
    "bplus256_point_all": dict(size="base_plus", image_size=256, T=4, n_cat=4, n_obj=3, prompt="point",
                               trainable=ALL),
    "bplus256_point_all_bf16": dict(size="base_plus", image_size=256, T=4, n_cat=4, n_obj=3, prompt="point",
                                    trainable=ALL, autocast="bf16"),
    # the loss knobs of the reference's experiments, applied as SAM2LightningModule.training_step
    # does: gt_stride 4 (trainer.py:190-203, sweeps/temp0.7+final_sweeps.yaml:5) with the
    # multi-step loss at logit temperature 0.7 (losses.py:166, configs/dice_loss_only.yaml:62)
    "bplus128_t8_gts4_temp07": dict(size="base_plus", image_size=128, T=8, n_cat=4, n_obj=3, prompt="point",
                                    trainable=ALL, loss=dict(kind="multistep", temperature=0.7, gt_stride=4)),
    # BCECategoryLoss (losses.py:251-372): 4 of 13 categories valid, temperature 0.7, mean
    "tiny256_point_all_bce": dict(size="tiny", image_size=256, T=4, n_cat=13, n_obj=4, prompt="point",
                                  trainable=ALL, loss=dict(kind="bce", temperature=0.7, reduction="mean")),
    # BCE with a per-category pos_weight (every category valid: the reference indexes pos_weight by
    # the valid set after checking its length against it, losses.py:348-363) and sum reduction
    "tiny256_bce_posw_sum": dict(size="tiny", image_size=256, T=3, n_cat=3, n_obj=3, prompt="point",
                                 trainable=ALL, loss=dict(kind="bce", temperature=1.0, reduction="sum",
                                                          pos_weight=[2.0, 0.5, 1.5])),
    # 8 frames at memory-attention Lq = 256 in fp32 and CPU bf16 autocast: the deep bank (7 memory
    # frames) and the frame-table flash backward over 7 frames, bf16 against the reference's bf16
    "bplus256_point_all_t8": dict(size="base_plus", image_size=256, T=8, n_cat=4, n_obj=3, prompt="point",
                                  trainable=ALL),
    # Hiera-L trunk (stages [2, 6, 36, 4], window_spec [8, 4, 16, 8], global blocks 23 / 33 / 43, head
    # dim 72, BASELINE config 4's model) at a small resolution
    "large128_point_all": dict(size="large", image_size=128, T=3, n_cat=4, n_obj=2, prompt="point", trainable=ALL),
    "bplus256_point_all_t8_bf16": dict(size="base_plus", image_size=256, T=8, n_cat=4, n_obj=3, prompt="point",
                                       trainable=ALL, autocast="bf16"),
}
FULL_GRAD_NUMEL = 4096


def reference_batch(clip):
    """Restates sam2_collate_fn (dataset.py:346-398) into the reference's BatchedVideoDatapoint."""
    from sam2_video.data.data_utils import BatchedVideoDatapoint, BatchedVideoMetaData

    images = clip["images"][:, None]  # [T, 1, 3, H, W]
    masks = clip["masks"]
    T, N = masks.shape[:2]
    H = images.shape[-2]
    obj_to_frame_idx = torch.zeros(T, N, 2, dtype=torch.int)
    obj_to_frame_idx[..., 0] = torch.arange(T, dtype=torch.int)[:, None]
    ident = torch.zeros(T, N, 3, dtype=torch.long)
    ident[..., 1] = torch.arange(N)[None]
    ident[..., 2] = torch.arange(T)[:, None]
    size = torch.full((T, N, 2), H, dtype=torch.long)
    meta = BatchedVideoMetaData(unique_objects_identifier=ident, frame_orig_size=size)
    return BatchedVideoDatapoint(img_batch=images, obj_to_frame_idx=obj_to_frame_idx, masks=masks.bool(),
                                 metadata=meta, dict_key="video_batch", batch_size=[T])


def run_case(name, c, seed=0, clip_idx=7):
    torch.manual_seed(0)
    model = H.build_reference_model(c["size"], c["image_size"], c["trainable"], c["prompt"], seed=seed)
    synth = H.product_file("data/synthetic.py")
    clip = synth.make_clip(clip_idx, c["T"], c["image_size"], c["n_cat"], c["n_obj"], c.get("parts"))
    batch = reference_batch(clip)
    from sam2_video.model.losses import BCECategoryLoss, MultiStepMultiMasksAndIous, CORE_LOSS_KEY
    from sam2_video.utils import merge_object_results_to_category

    lc = c.get("loss", {})
    if lc.get("kind") == "bce":
        crit = BCECategoryLoss(pos_weight=lc.get("pos_weight"), reduction=lc.get("reduction", "mean"),
                               logit_temperature=lc.get("temperature", 1.0))
    else:
        crit = MultiStepMultiMasksAndIous(weight_dict={"loss_mask": 20, "loss_dice": 1, "loss_iou": 1,
                                                       "loss_class": 0},
                                          supervise_all_iou=True, iou_use_l1_loss=True, pred_obj_scores=False,
                                          focal_gamma_obj_score=0.0, focal_alpha_obj_score=-1.0,
                                          logit_temperature=lc.get("temperature", 1.0))
    gt_stride = int(lc.get("gt_stride", 1))
    t0 = time.time()
    # SAM2Model.forward (sam2model.py:153-179), restated to keep the per-object outputs; under
    # `autocast` the forward + loss run in torch.autocast("cpu", bfloat16) (the reference's
    # trainer.precision bf16-mixed), the backward outside it as Lightning does
    import contextlib
    ac = (torch.autocast("cpu", dtype=torch.bfloat16) if c.get("autocast") == "bf16"
          else contextlib.nullcontext())
    with ac:
        backbone_out = model.forward_image(batch.flat_img_batch)
        feats = {f"fpn{i}": x.detach().float().clone() for i, x in enumerate(backbone_out["backbone_fpn"])}
        backbone_out = model.prepare_prompt_inputs(backbone_out, batch)
        stages = model.forward_tracking(backbone_out, batch)
        outs = merge_object_results_to_category(stages, backbone_out["obj_to_cat"],
                                                backbone_out["num_categories"])
        # SAM2LightningModule._apply_gt_stride (trainer.py:190-203), restated: Lightning is absent
        if gt_stride > 1:
            idxs = list(range(0, len(outs), gt_stride))
            losses = crit([outs[i] for i in idxs], batch.masks[idxs])
        else:
            losses = crit(outs, batch.masks)
    total = losses[CORE_LOSS_KEY]
    total.backward()
    dt = time.time() - t0

    g = {}
    g["meta/T"] = torch.tensor(c["T"])
    g["meta/image_size"] = torch.tensor(c["image_size"])
    g["meta/seed"] = torch.tensor(seed)
    g["meta/clip_idx"] = torch.tensor(clip_idx)
    g["meta/parts"] = torch.tensor(list(c.get("parts") or []), dtype=torch.long)
    g["meta/autocast"] = torch.tensor(1 if c.get("autocast") == "bf16" else 0)
    g["meta/loss_kind"] = lc.get("kind", "multistep")
    g["meta/temperature"] = torch.tensor(float(lc.get("temperature", 1.0)))
    g["meta/gt_stride"] = torch.tensor(gt_stride)
    g["meta/reduction"] = lc.get("reduction", "mean")
    if lc.get("pos_weight") is not None:
        g["meta/pos_weight"] = torch.tensor(lc["pos_weight"], dtype=torch.float32)
    g["in/images_sum"] = clip["images"].double().sum()
    g["in/images_abs"] = clip["images"].double().abs().sum()
    g["in/masks_count"] = clip["masks"].sum(dim=(2, 3))
    g["obj_to_cat"] = torch.tensor(backbone_out["obj_to_cat"])
    pin = backbone_out["point_inputs_per_frame"].get(0)
    if pin is not None:
        g["prompt/coords"] = pin["point_coords"].detach().clone()
        g["prompt/labels"] = pin["point_labels"].detach().clone()
    for k, v in feats.items():
        g[f"feat/{k}_sum"] = v.double().sum()
        g[f"feat/{k}_sq"] = (v.double() ** 2).sum()
    g["feat/fpn_last"] = feats[f"fpn{len(feats) - 1}"]
    for t, st in enumerate(stages):
        g[f"obj/{t}/low_res"] = st["pred_masks"].detach().float().clone()
        g[f"obj/{t}/ious"] = st["multistep_pred_ious"][0].detach().float().clone()
        g[f"obj/{t}/obj_score"] = st["multistep_object_score_logits"][0].detach().float().clone()
    for t, o in enumerate(outs):
        hr = o["multistep_pred_multimasks_high_res"][0].detach().float()
        g[f"cat/{t}/low_res"] = o["pred_masks"].detach().float().clone()
        g[f"cat/{t}/high_res_sub"] = hr[:, :, ::8, ::8].clone()
        g[f"cat/{t}/high_res_sum"] = hr.double().sum()
        g[f"cat/{t}/high_res_sq"] = (hr.double() ** 2).sum()
        g[f"cat/{t}/ious"] = o["multistep_pred_ious"][0].detach().float().clone()
        g[f"cat/{t}/obj_score"] = o["multistep_object_score_logits"][0].detach().float().clone()
    for k in [k for k in losses if k != "logits"]:
        v = losses[k]
        g[f"loss/{k}"] = v.detach().float().clone() if torch.is_tensor(v) else torch.tensor(float(v))
    none_grad = []
    for n, p in model.named_parameters():
        if not p.requires_grad:
            continue
        if p.grad is None:
            none_grad.append(n)
            continue
        g[f"gnorm/{n}"] = p.grad.double().norm()
        g[f"gsum/{n}"] = p.grad.double().sum()
        if p.numel() <= FULL_GRAD_NUMEL:
            g[f"grad/{n}"] = p.grad.detach().clone()
    g["none_grad"] = none_grad
    g["trainable"] = [n for n, p in model.named_parameters() if p.requires_grad]
    g["state_shapes"] = {k: list(v.shape) for k, v in model.state_dict().items()}
    path = os.path.join(OUT, f"{name}.pt")
    torch.save(g, path)
    print(f"{name}: step {dt:.1f}s, loss {float(total):.6f}, {len(none_grad)} none-grad params, "
          f"{os.path.getsize(path) / 1e6:.2f} MB")


def main(argv):
    os.makedirs(OUT, exist_ok=True)
    names = argv or list(CASES)
    for n in names:
        run_case(n, CASES[n])


if __name__ == "__main__":
    main(sys.argv[1:])
