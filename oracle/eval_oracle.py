"""TEST INFRASTRUCTURE ONLY -- CPU restatement of the reference's evaluation metrics
(sam2_video/eval/eval.py), the checker for sam2_video.eval on the GPU.  Only tests/ and
bench.py's checks may import this file; the product never does.  Pinned against the
reference itself through tests/golden/eval_small.pt (oracle/gen_eval_golden.py runs the
reference's get_image_scores / get_video_scores / get_result) in tests/test_eval.py.
"""
from __future__ import annotations

import numpy as np

KEYS = ("iou", "mae", "dice")


def nanmean(v):
    v = np.asarray(v, dtype=np.float64)
    return float(np.nanmean(v)) if v.size and not np.all(np.isnan(v)) else float("nan")


def image_scores(pred_bin, gt, cat_ids=None):
    """get_image_scores (eval/eval.py:53-141) for one frame, on masks instead of COCO
    annotations: pred_bin / gt [N_cat, H, W] bool.  A category has a detection (resp. ground
    truth) annotation iff its mask is non-empty (inference.py:887-889 skips empty predicted
    masks, convert_endovis_to_coco.py:150 empty ground truth); categories with neither are
    skipped (:85-86) and read NaN.  iou / mae / dice: caculate_iou / _mae / _dice (:16-40)."""
    pred_bin = np.asarray(pred_bin, dtype=bool)
    gt = np.asarray(gt, dtype=bool)
    cat_ids = list(range(pred_bin.shape[0])) if cat_ids is None else list(cat_ids)
    cat = {}
    for n, c in enumerate(cat_ids):
        p, g = pred_bin[n], gt[n]
        if not p.any() and not g.any():
            cat[c] = {k: float("nan") for k in KEYS}
            continue
        pu, gu = p.astype(np.uint8), g.astype(np.uint8)
        inter = np.logical_and(pu, gu).sum()
        iou = inter / (np.logical_or(pu, gu).sum() + 1e-7)
        # caculate_mae(merged_dt, merged_gt) runs on uint8 masks (eval.py:39-40, :50, :102):
        # dt - gt wraps to 255 where dt = 0 and gt = 1
        mae = np.mean(np.abs(pu - gu))
        dice = (2.0 * np.sum(pu * gu)) / (np.sum(pu) + np.sum(gu) + 1e-7)
        cat[c] = {"iou": float(iou), "mae": float(mae), "dice": float(dice)}
    return {"cat_scores": cat, "avg_scores": {k: nanmean([cat[c][k] for c in cat_ids]) for k in KEYS}}


def video_scores(img_scores, cat_ids):
    """get_video_scores (eval/eval.py:144-206) for one video: per category nanmean over its
    frames, then nanmean over categories."""
    cat = {c: {k: nanmean([f["cat_scores"][c][k] for f in img_scores]) for k in KEYS} for c in cat_ids}
    return {"cat_scores": cat, "avg_scores": {k: nanmean([cat[c][k] for c in cat_ids]) for k in KEYS}}


def result(videos, cat_ids):
    """get_result (eval/eval.py:209-258): per category nanmean over videos, then over categories."""
    return video_scores(videos, cat_ids)
