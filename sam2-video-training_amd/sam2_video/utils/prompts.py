"""Prompt generation (reference sam2_video/utils/prompts.py:13-97), host-side,
once per clip on the frame-0 object masks."""
from __future__ import annotations

from typing import Tuple

import numpy as np
import torch
from scipy import ndimage


def generate_point_prompt(mask: torch.Tensor, num_pos_points: int = 1, num_neg_points: int = 0,
                          include_center: bool = True) -> Tuple[torch.Tensor, torch.Tensor]:
    """[B, 1, H, W] -> points [B, P, 2] (x, y) f32, labels [B, P] int32 (prompts.py:13-75)"""
    B = mask.shape[0]
    m_all = (mask.detach().cpu().squeeze(1) > 0).to(torch.uint8)
    total = num_pos_points + num_neg_points
    points = torch.empty(B, total, 2, dtype=torch.float32)
    labels = torch.empty(B, total, dtype=torch.int32)
    for b in range(B):
        m = m_all[b]
        pos_coords = torch.stack(torch.where(m == 1), dim=1)
        n_pos = pos_coords.shape[0]
        if num_pos_points > 0 and n_pos == 0:
            raise ValueError("generate_point_prompt: no positive pixels available for sampling")
        pts = []
        if n_pos > 0 and include_center and num_pos_points > 0:
            cy, cx = ndimage.center_of_mass(m.numpy())
            pts.append(torch.tensor([[cx, cy]], dtype=torch.float32))
            need = max(0, num_pos_points - 1)
        else:
            need = num_pos_points
        if need > 0:
            idx = torch.randperm(n_pos)[:need]
            pts.append(pos_coords[idx].flip(-1).float())
        pos_pts = torch.cat(pts, 0) if num_pos_points > 0 else torch.empty(0, 2)
        neg_coords = torch.stack(torch.where(m == 0), dim=1)
        if num_neg_points > 0 and neg_coords.shape[0] > 0:
            idx = torch.randperm(neg_coords.shape[0])[:num_neg_points]
            neg_pts = neg_coords[idx].flip(-1).float()
        else:
            neg_pts = torch.empty(0, 2)
        points[b] = torch.cat([pos_pts, neg_pts], 0)
        labels[b] = torch.cat([torch.ones(pos_pts.shape[0], dtype=torch.int32),
                               torch.zeros(neg_pts.shape[0], dtype=torch.int32)])
    return points, labels


def generate_box_prompt(mask: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """bounding-box corners as clicks with labels 2 / 3 (prompts.py:78-97)"""
    B = mask.shape[0]
    points = torch.empty((B, 2, 2), dtype=torch.float32)
    labels = torch.empty((B, 2), dtype=torch.int32)
    mc = mask.detach().cpu()
    for i in range(B):
        ys, xs = np.where(mc[i, 0].numpy() > 0)
        if xs.size == 0:
            raise ValueError("generate_box_prompt: no positive pixels to form a bounding box")
        points[i, 0] = torch.tensor([float(xs.min()), float(ys.min())])
        points[i, 1] = torch.tensor([float(xs.max()), float(ys.max())])
        labels[i, 0], labels[i, 1] = 2, 3
    return points, labels
