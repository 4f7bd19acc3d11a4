"""Evaluation metrics -- drop-in for sam2_video/eval/eval.py of the reference (IoU / Dice / MAE
of the category-merged binarised masks, aggregated per frame, per video and over videos).

The reference evaluates offline from COCO json (predictions written by inference.py:862-901,
one annotation per non-empty merged category mask).  Here the same numbers are computed in
the loop from the model's outputs: one HIP reduction per frame (s2h_mask_eval_counts) gives
|pred & gt|, |pred | gt|, |pred|, |gt| per category on the device, and the scores follow in
closed form from those integers:
    iou  = |p & g| / (|p | g| + 1e-7)                     caculate_iou   (eval.py:16-30)
    dice = 2 |p & g| / (|p| + |g| + 1e-7)                 caculate_dice  (eval.py:33-36)
    mae  = (|p & !g| + 255 |!p & g|) / P                  caculate_mae(dt, gt) on uint8
                                                          masks (eval.py:39-40, :102): dt - gt
                                                          wraps to 255 where dt = 0, gt = 1
A category with neither a predicted nor a ground-truth pixel has no annotation in either file
and is skipped (eval.py:85-86) -- NaN, ignored by the nanmeans.  The per-video and overall
aggregation (get_video_scores / get_result) is nanmean over at most a few dozen numbers, done on
the host.  The numpy helpers keep the reference's names and signatures.
"""
from __future__ import annotations

from typing import Dict, List, Sequence

import numpy as np
import torch

from ..kernels import ops

KEYS = ("iou", "mae", "dice")


# ---------------------------------------------------------- reference helpers (host, numpy)
def caculate_iou(pred, gt):
    """eval.py:16-30"""
    intersection = np.logical_and(pred, gt).sum()
    union = np.logical_or(pred, gt).sum() + 1e-7
    return intersection / union


def caculate_dice(pred, gt):
    """eval.py:33-36"""
    intersection = np.sum(pred * gt)
    return (2.0 * intersection) / (np.sum(pred) + np.sum(gt) + 1e-7)


def caculate_mae(y_true, y_pred):
    """eval.py:39-40"""
    return np.mean(np.abs(y_true - y_pred))


def merge_masks(masks):
    """eval.py:43-50"""
    if not masks:
        return None
    merged = np.zeros_like(masks[0])
    for m in masks:
        merged = np.logical_or(merged, m)
    return merged.astype(np.uint8)


def _nanmean(v):
    v = np.asarray(v, dtype=np.float64)
    return float(np.nanmean(v)) if v.size and not np.all(np.isnan(v)) else float("nan")


# ------------------------------------------------------------------ device path
def frame_counts(pred_logits: torch.Tensor, gt: torch.Tensor) -> torch.Tensor:
    """[N_cat, 4] int64 on the device: |p & g|, |p | g|, |p|, |g| with p = pred_logits > 0.
    pred_logits [N_cat, (1,) H, W] fp32 (category-merged high-res logits), gt [N_cat, H, W]."""
    return ops.mask_eval_counts(pred_logits.detach().contiguous(), gt.contiguous())


def image_scores_from_counts(counts, num_pixels: int, cat_ids: Sequence = None) -> Dict:
    """get_image_scores (eval.py:53-141) for one frame from the per-category counts."""
    c = np.asarray(counts, dtype=np.int64).reshape(-1, 4)
    cat_ids = list(range(c.shape[0])) if cat_ids is None else list(cat_ids)
    cat = {}
    for n, cid in enumerate(cat_ids):
        inter, union, npred, ngt = (int(v) for v in c[n])
        if npred == 0 and ngt == 0:
            cat[cid] = {k: float("nan") for k in KEYS}
            continue
        cat[cid] = {"iou": inter / (union + 1e-7),
                    "mae": ((npred - inter) + 255.0 * (ngt - inter)) / float(num_pixels),
                    "dice": (2.0 * inter) / (npred + ngt + 1e-7)}
    return {"cat_scores": cat, "avg_scores": {k: _nanmean([cat[i][k] for i in cat_ids]) for k in KEYS}}


def get_video_scores_from_frames(img_scores: List[Dict], cat_ids: Sequence) -> Dict:
    """get_video_scores (eval.py:144-206) for one video"""
    cat = {c: {k: _nanmean([f["cat_scores"][c][k] for f in img_scores]) for k in KEYS} for c in cat_ids}
    return {"frames": img_scores, "cat_scores": cat,
            "avg_scores": {k: _nanmean([cat[c][k] for c in cat_ids]) for k in KEYS}}


def get_result(video_scores: List[Dict], cat_ids: Sequence) -> Dict:
    """get_result (eval.py:209-258)"""
    cat = {c: {k: _nanmean([v["cat_scores"][c][k] for v in video_scores]) for k in KEYS} for c in cat_ids}
    return {"videos": video_scores, "cat_scores": cat,
            "avg_scores": {k: _nanmean([cat[c][k] for c in cat_ids]) for k in KEYS}}


@torch.no_grad()
def evaluate_clip(merged_frames: List[Dict], target_masks: torch.Tensor, cat_ids: Sequence = None) -> Dict:
    """Scores of one clip from SAM2Model.forward's category-merged outputs (pred_masks_high_res
    [N_cat, 1, H, W] per frame) against its masks [T, N_cat, H, W]: the video-level dict of
    get_video_scores, every frame counted (synthetic clips have no non-keyframes)."""
    T = len(merged_frames)
    counts = torch.stack([frame_counts(f["pred_masks_high_res"], target_masks[t]) for t, f in enumerate(merged_frames)])
    counts = counts.cpu().numpy()  # one device->host copy per clip
    n_cat = counts.shape[1]
    cat_ids = list(range(n_cat)) if cat_ids is None else list(cat_ids)
    P = int(target_masks[0, 0].numel())
    frames = [image_scores_from_counts(counts[t], P, cat_ids) for t in range(T)]
    return get_video_scores_from_frames(frames, cat_ids)
