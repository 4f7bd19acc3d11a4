"""Object/category mask utilities (reference sam2_video/utils/masks.py).

* find_connected_components / cat_to_obj_mask (masks.py:13-50): host-side, once
  per clip on frame 0 -- the 5x5 ellipse opening (erode with +inf border,
  dilate with -inf border) and 8-connected labelling in raster order -- in the
  library's native host code (csrc/prompts_host.cpp: separable byte passes and a
  union-find labelling, one thread per category).  `object_moments` gives the
  objects' categories and moments without materialising their masks (the point
  and box prompts need only those).
* merge_object_results_to_category (masks.py:53-213): on the device -- pixelwise
  max over a category's objects for mask logits, sigmoid-mass weighted mean for
  IoU / object-score predictions (differentiable in the weights too).
"""
from __future__ import annotations

import ctypes
import os
from typing import Any, Dict, List, Tuple

import numpy as np
import torch

N_STATS = 7  # count, sum_y, sum_x, y_min, y_max, x_min, x_max
_THREADS = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else 4))


def _u8(m) -> np.ndarray:
    """0/1 bytes, C-contiguous, of a bool / numeric mask (tensor or array)"""
    if isinstance(m, torch.Tensor):
        m = m.detach().cpu()
        m = (m if m.dtype == torch.bool else m > 0).numpy()
    else:
        m = np.asarray(m)
        m = m if m.dtype == np.bool_ else m > 0
    return np.ascontiguousarray(m).view(np.uint8)


def object_moments(cat_masks, want_labels: bool = False):
    """N category masks [N, H, W] -> (obj_cat int32 [O], stats int64 [O, 7], labels int32
    [N, H, W] or None): the objects of cat_to_obj_mask (opening + 8-connected components,
    category-major, raster order) and their moments."""
    from ..kernels import _lib
    m = _u8(cat_masks)
    N, H, W = m.shape
    lab = np.empty((N, H, W), np.int32) if want_labels else None
    cap = 64
    while True:
        n = ctypes.c_int(0)
        cats = np.empty(cap, np.int32)
        stats = np.empty((cap, N_STATS), np.int64)
        rc = _lib.host_lib().s2h_prompt_objects(N, H, W, m.ctypes.data, cap, ctypes.byref(n), cats.ctypes.data,
                                                stats.ctypes.data, lab.ctypes.data if lab is not None else None, _THREADS)
        if rc == 2:
            cap = n.value
            continue
        if rc != 0:
            raise ValueError(f"s2h_prompt_objects: bad arguments (rc {rc}) for masks of shape {m.shape}")
        return cats[:n.value], stats[:n.value], lab


def object_masks(labels: np.ndarray, n_obj: int) -> torch.Tensor:
    """labels of object_moments -> float object masks [O, H, W]"""
    from ..kernels import _lib
    N, H, W = labels.shape
    out = torch.empty(n_obj, H, W, dtype=torch.float32)
    _lib.host_call("s2h_prompt_object_masks", N, H, W, labels.ctypes.data, n_obj, out.data_ptr(), _THREADS)
    return out


def mask_moments(masks) -> np.ndarray:
    """B whole masks [B, H, W] -> int64 [B, 7] moments (no opening)"""
    from ..kernels import _lib
    m = _u8(masks)
    B, H, W = m.shape
    stats = np.empty((B, N_STATS), np.int64)
    _lib.host_call("s2h_mask_moments", B, H, W, m.ctypes.data, stats.ctypes.data, _THREADS)
    return stats


def find_connected_components(mask: torch.Tensor) -> List[torch.Tensor]:
    """masks.py:13-28: the opened mask's 8-connected components, raster order, as float masks"""
    m = _u8(mask)
    _, stats, lab = object_moments(m[None], want_labels=True)
    return list(object_masks(lab, len(stats)).unbind(0))


def cat_to_obj_mask(cat_frame_masks: torch.Tensor) -> Tuple[torch.Tensor, List[int], int]:
    """[N, 1, H, W] category masks -> ([O, 1, H, W] float object masks (host), obj_to_cat, N)"""
    N = int(cat_frame_masks.shape[0])
    cats, stats, lab = object_moments(_u8(cat_frame_masks)[:, 0], want_labels=True)
    if len(cats) == 0:
        raise ValueError("cat_to_obj_mask: no objects found in category masks (fail-fast)")
    return object_masks(lab, len(cats)).unsqueeze(1), cats.tolist(), N


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
    from ..kernels.functional_sam import merge_masks, merge_masks_scores, merge_scores_stats

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
        # the high-res masks and the IoU scores weighted by them as one autograd node
        m["pred_masks_high_res"], merged_ious, hr_stats = merge_masks_scores(hr, fo["multistep_pred_ious"][0], groups)
        with torch.no_grad():
            m["pred_masks"] = merge_masks(fo["pred_masks"].detach(), groups)
        m["multistep_pred_masks"] = m["pred_masks"]
        m["multistep_pred_masks_high_res"] = m["pred_masks_high_res"]
        m["multistep_pred_multimasks"] = [m["pred_masks"]]
        m["multistep_pred_multimasks_high_res"] = [m["pred_masks_high_res"]]
        m["multistep_pred_ious"] = [merged_ious]
        with torch.no_grad():
            # weighted by the same high-res statistics (computed once, above)
            m["multistep_object_score_logits"] = [merge_scores_stats(fo["multistep_object_score_logits"][0],
                                                                     hr_stats, groups)]
        m["point_inputs"] = fo.get("point_inputs")
        m["mask_inputs"] = fo.get("mask_inputs")
        m["multistep_point_inputs"] = [None]
        merged_all.append(m)
    return merged_all
