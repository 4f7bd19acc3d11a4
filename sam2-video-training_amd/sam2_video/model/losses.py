"""Losses (reference sam2_video/model/losses.py).

MultiStepMultiMasksAndIous: per frame, one fused reduction kernel over the
category-level high-res logits (focal + sigmoid sums + IoU counts), a finalize
kernel (valid-category filter, Dice, IoU-L1, weighted total, backward
coefficients) and, in backward, one elementwise kernel producing dlogits and
d(pred IoU).  The single-mask path (loss_multimask.size(1) == 1) is the one the
training step takes (multimask_output=False).
"""
from __future__ import annotations

from typing import Dict, List

import torch
from torch import nn

from ..kernels import functional as FN
from ..kernels.functional_sam import bce_frame_loss, clip_loss

CORE_LOSS_KEY = "total_loss"


class MultiStepMultiMasksAndIous(nn.Module):
    def __init__(self, weight_dict, focal_alpha=0.25, focal_gamma=2.0, supervise_all_iou=False,
                 iou_use_l1_loss=False, pred_obj_scores=False, focal_gamma_obj_score=0.0, focal_alpha_obj_score=-1,
                 logit_temperature: float = 1.0):
        super().__init__()
        self.weight_dict = dict(weight_dict)
        assert "loss_mask" in self.weight_dict and "loss_dice" in self.weight_dict and "loss_iou" in self.weight_dict
        self.weight_dict.setdefault("loss_class", 0.0)
        if focal_alpha != 0.25 or focal_gamma != 2.0 or not iou_use_l1_loss or pred_obj_scores:
            raise NotImplementedError("kernels implement alpha=.25, gamma=2, L1 IoU loss, pred_obj_scores=False "
                                      "(the reference training configs)")
        if float(self.weight_dict["loss_class"]) != 0.0:
            raise NotImplementedError("loss_class weight must be 0 with pred_obj_scores=False")
        if not (isinstance(logit_temperature, (int, float)) and logit_temperature > 0):
            raise ValueError("logit_temperature must be a positive float")
        self.supervise_all_iou = supervise_all_iou
        self.logit_temperature = float(logit_temperature)

    def forward(self, outs_batch: List[Dict], targets_batch: torch.Tensor) -> Dict[str, torch.Tensor]:
        """losses.py:111-121: sum over frames of the per-frame weighted losses"""
        assert len(outs_batch) == len(targets_batch)
        w = (float(self.weight_dict["loss_mask"]), float(self.weight_dict["loss_dice"]),
             float(self.weight_dict["loss_iou"]))
        # every frame's losses accumulated into one buffer by one autograd node (FN clip_loss)
        acc = clip_loss([(outs["multistep_pred_multimasks_high_res"][0], outs["multistep_pred_ious"][0],
                          targets.contiguous()) for outs, targets in zip(outs_batch, targets_batch)],
                        w, self.logit_temperature)
        losses = {"loss_mask": acc[0], "loss_dice": acc[1], "loss_iou": acc[2],
                  "loss_class": torch.zeros((), device=acc.device), CORE_LOSS_KEY: acc[3]}
        return losses


class BCECategoryLoss(nn.Module):
    """losses.py:251-372: per frame, binary_cross_entropy_with_logits(logits / T, gt, pos_weight)
    over the categories that have ground-truth pixels (category-level `pred_masks_high_res`,
    else `pred_masks`), "mean" or "sum" reduction, averaged over frames.  One statistics kernel,
    one finalize kernel and, in backward, one elementwise kernel per frame."""

    def __init__(self, pos_weight=None, reduction: str = "mean", logit_temperature: float = 1.0):
        super().__init__()
        if isinstance(pos_weight, (list, tuple)):
            pos_weight = torch.tensor(pos_weight, dtype=torch.float32)
        self._pos_weight = pos_weight.float().reshape(-1) if isinstance(pos_weight, torch.Tensor) else None
        if reduction not in ("mean", "sum"):
            raise NotImplementedError("BCECategoryLoss reductions: mean | sum (the per-frame sum of a 'none' "
                                      "reduction is not shape-stable in the reference either)")
        self.reduction = reduction
        if not (isinstance(logit_temperature, (int, float)) and logit_temperature > 0):
            raise ValueError("logit_temperature must be a positive float")
        self.logit_temperature = float(logit_temperature)

    def forward(self, outs_batch: List[Dict], targets_batch: torch.Tensor) -> Dict[str, torch.Tensor]:
        assert len(outs_batch) == len(targets_batch), (
            f"Mismatched sequence lengths: outs={len(outs_batch)} vs targets={len(targets_batch)}")
        num_frames = len(outs_batch)
        acc = None
        for outs, targets in zip(outs_batch, targets_batch):
            logits = outs.get("pred_masks_high_res")
            if logits is None:
                logits = outs.get("pred_masks")
            if logits is None:
                raise KeyError("BCECategoryLoss expects 'pred_masks_high_res' or 'pred_masks' in outputs")
            if logits.dim() == 4 and logits.shape[1] == 1:
                logits = logits.squeeze(1)
            elif logits.dim() != 3:
                raise ValueError(f"Unexpected logits shape for BCECategoryLoss: {tuple(logits.shape)}")
            if targets.dim() != 3:
                raise ValueError(f"Unexpected target shape for BCECategoryLoss: {tuple(targets.shape)}")
            pw = None
            if self._pos_weight is not None:
                if self._pos_weight.numel() != logits.shape[0]:
                    raise ValueError(f"pos_weight length {self._pos_weight.numel()} does not match number of "
                                     f"classes {logits.shape[0]}")
                pw = self._pos_weight.to(logits.device)
            lf = bce_frame_loss(logits.float().contiguous(), targets.contiguous(), pw, self.logit_temperature,
                                0 if self.reduction == "mean" else 1, 1.0 / max(num_frames, 1))
            acc = lf if acc is None else FN.add(acc, lf)
        total = acc[0]
        return {"loss_bce": total, CORE_LOSS_KEY: total}
