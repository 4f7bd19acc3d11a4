"""Object/category mask utilities (reference sam2_video/utils/masks.py).

* find_connected_components / cat_to_obj_mask (masks.py:13-50): host-side, once
  per clip on frame 0 -- the 5x5 ellipse opening (erode with +inf border,
  dilate with -inf border) and 8-connected labelling in raster order, restated
  on scipy.ndimage (cv2 is not a dependency of this build).
* merge_object_results_to_category (masks.py:53-213): on the device -- pixelwise
  max over a category's objects for mask logits, sigmoid-mass weighted mean for
  IoU / object-score predictions (differentiable in the weights too).
"""
from __future__ import annotations

from typing import Any, Dict, List, Tuple

import numpy as np
import torch
from scipy import ndimage

_ELLIPSE5 = np.ones((5, 5), bool)
_ELLIPSE5[0, [0, 1, 3, 4]] = False
_ELLIPSE5[4, [0, 1, 3, 4]] = False


def find_connected_components(mask: torch.Tensor) -> List[torch.Tensor]:
    m = mask.detach().cpu().numpy().astype(bool)
    m = ndimage.binary_erosion(m, structure=_ELLIPSE5, border_value=1)
    m = ndimage.binary_dilation(m, structure=_ELLIPSE5, border_value=0)
    lab, n = ndimage.label(m, structure=np.ones((3, 3), int))
    return [torch.from_numpy((lab == i).astype(np.float32)) for i in range(1, n + 1)]


def cat_to_obj_mask(cat_frame_masks: torch.Tensor) -> Tuple[torch.Tensor, List[int], int]:
    """[N, 1, H, W] category masks -> ([O, 1, H, W] float object masks (host), obj_to_cat, N)"""
    N = int(cat_frame_masks.shape[0])
    cm = cat_frame_masks.detach().cpu()
    obj_to_cat, objs = [], []
    for c in range(N):
        m = cm[c][0] > 0
        if not bool(m.any()):
            continue
        for comp in find_connected_components(m):
            objs.append(comp)
            obj_to_cat.append(c)
    if not objs:
        raise ValueError("cat_to_obj_mask: no objects found in category masks (fail-fast)")
    return torch.stack(objs).unsqueeze(1), obj_to_cat, N


_GROUP_CACHE = {}


class CategoryGroups:
    """device index lists of the object -> category grouping for the merge kernels"""

    def __init__(self, obj_to_cat: List[int], num_categories: int, device):
        groups = [[] for _ in range(num_categories)]
        for o, c in enumerate(obj_to_cat):
            groups[int(c)].append(o)
        off = [0]
        flat = []
        for g in groups:
            flat += g
            off.append(len(flat))
        self.ncat = num_categories
        self.cat_off = torch.tensor(off, dtype=torch.int32, device=device)
        self.cat_obj = torch.tensor(flat if flat else [0], dtype=torch.int32, device=device)
        self.obj_cat = torch.tensor(list(obj_to_cat), dtype=torch.int32, device=device)


def merge_object_results_to_category(previous_stages_out: List[Dict[str, Any]], obj_to_cat: List[int],
                                     num_categories: int) -> List[Dict[str, Any]]:
    """masks.py:53-213 for the per-frame outputs of forward_tracking."""
    from ..kernels.functional_sam import merge_masks, merge_scores

    if not previous_stages_out:
        return []
    dev = previous_stages_out[0]["pred_masks_high_res"].device
    key = (tuple(obj_to_cat), num_categories, str(dev))
    groups = _GROUP_CACHE.get(key)
    if groups is None:
        groups = _GROUP_CACHE[key] = CategoryGroups(obj_to_cat, num_categories, dev)
    merged_all = []
    for fo in previous_stages_out:
        hr = fo["pred_masks_high_res"]
        m = {}
        m["pred_masks_high_res"] = merge_masks(hr, groups)
        with torch.no_grad():
            m["pred_masks"] = merge_masks(fo["pred_masks"].detach(), groups)
        m["multistep_pred_masks"] = m["pred_masks"]
        m["multistep_pred_masks_high_res"] = m["pred_masks_high_res"]
        m["multistep_pred_multimasks"] = [m["pred_masks"]]
        m["multistep_pred_multimasks_high_res"] = [m["pred_masks_high_res"]]
        m["multistep_pred_ious"] = [merge_scores(fo["multistep_pred_ious"][0], hr, groups)]
        with torch.no_grad():
            m["multistep_object_score_logits"] = [merge_scores(fo["multistep_object_score_logits"][0], hr.detach(),
                                                               groups)]
        m["point_inputs"] = fo.get("point_inputs")
        m["mask_inputs"] = fo.get("mask_inputs")
        m["multistep_point_inputs"] = [None]
        merged_all.append(m)
    return merged_all
