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
from ..kernels.functional_sam import frame_loss

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
        acc = None
        for outs, targets in zip(outs_batch, targets_batch):
            src = outs["multistep_pred_multimasks_high_res"][0]
            ious = outs["multistep_pred_ious"][0]
            lt = frame_loss(src, ious, targets.contiguous(), None, w, self.logit_temperature)
            acc = lt if acc is None else FN.add(acc, lt)
        losses = {"loss_mask": acc[0], "loss_dice": acc[1], "loss_iou": acc[2],
                  "loss_class": torch.zeros((), device=acc.device), CORE_LOSS_KEY: acc[3]}
        return losses


class BCECategoryLoss(nn.Module):
    def __init__(self, pos_weight=None, reduction: str = "mean", logit_temperature: float = 1.0):
        super().__init__()
        raise NotImplementedError("BCECategoryLoss (loss.type=bce) is not built yet in this MI355X build")
