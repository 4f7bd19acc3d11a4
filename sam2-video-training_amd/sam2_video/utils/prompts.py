"""Prompt generation (reference sam2_video/utils/prompts.py:13-97), host-side,
once per clip on the frame-0 object masks.  Centres of mass and boxes come from
the native mask moments (masks.mask_moments); only random clicks scan pixels."""
from __future__ import annotations

from typing import Tuple

import torch

from .masks import mask_moments


def generate_point_prompt(mask: torch.Tensor, num_pos_points: int = 1, num_neg_points: int = 0,
                          include_center: bool = True) -> Tuple[torch.Tensor, torch.Tensor]:
    """[B, 1, H, W] -> points [B, P, 2] (x, y) f32, labels [B, P] int32 (prompts.py:13-75)"""
    B = mask.shape[0]
    m_all = (mask.detach().cpu().squeeze(1) > 0)
    st = mask_moments(m_all)
    total = num_pos_points + num_neg_points
    points = torch.empty(B, total, 2, dtype=torch.float32)
    labels = torch.empty(B, total, dtype=torch.int32)
    for b in range(B):
        m = m_all[b]
        n_pos = int(st[b, 0])
        if num_pos_points > 0 and n_pos == 0:
            raise ValueError("generate_point_prompt: no positive pixels available for sampling")
        pts = []
        if n_pos > 0 and include_center and num_pos_points > 0:
            # centre of mass (x, y) = float64 mean of the pixel coordinates (ndimage.center_of_mass)
            pts.append(torch.tensor([[st[b, 2] / st[b, 0], st[b, 1] / st[b, 0]]], dtype=torch.float32))
            need = max(0, num_pos_points - 1)
        else:
            need = num_pos_points
        if need > 0:
            pos_coords = torch.stack(torch.where(m), dim=1)
            idx = torch.randperm(n_pos)[:need]
            pts.append(pos_coords[idx].flip(-1).float())
        pos_pts = torch.cat(pts, 0) if num_pos_points > 0 else torch.empty(0, 2)
        neg_coords = torch.stack(torch.where(~m), dim=1) if num_neg_points > 0 else None
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
    return box_prompt_from_moments(mask_moments(mask.detach().cpu()[:, 0]))


def box_prompt_from_moments(st) -> Tuple[torch.Tensor, torch.Tensor]:
    """[B, 7] moments -> corners (x_min, y_min), (x_max, y_max), labels 2 / 3"""
    B = st.shape[0]
    if B and int(st[:, 0].min()) == 0:
        raise ValueError("generate_box_prompt: no positive pixels to form a bounding box")
    st = torch.as_tensor(st)
    points = torch.stack([st[:, [5, 3]], st[:, [6, 4]]], dim=1).float()
    labels = torch.tensor([[2, 3]], dtype=torch.int32).expand(B, 2).contiguous()
    return points, labels


def center_prompt_from_moments(st) -> Tuple[torch.Tensor, torch.Tensor]:
    """[B, 7] moments -> generate_point_prompt(num_pos_points=1, num_neg_points=0,
    include_center=True): one click at the centre of mass, label 1"""
    B = st.shape[0]
    if B and int(st[:, 0].min()) == 0:
        raise ValueError("generate_point_prompt: no positive pixels available for sampling")
    st = torch.as_tensor(st).double()
    points = torch.stack([st[:, 2] / st[:, 0], st[:, 1] / st[:, 0]], dim=1).float().unsqueeze(1)
    return points, torch.ones(B, 1, dtype=torch.int32)
