"""Deterministic synthetic clips of the benchmark shapes and the
clip collate function (restates sam2_collate_fn, reference
sam2_video/data/dataset.py:346-398, B == 1 enforced).

Images ~ N(0, 1) (already "normalised"), seeded by clip index.  Masks: category
c < n_obj holds one disc of radius cell/4 centred in grid cell c (grid =
ceil(sqrt(n_cat)), cell = H // grid), drifting (+1, +1) px per frame; the other
categories are empty.  Every disc survives the 5x5 opening, so the number of
tracked objects equals n_obj.

This file depends on torch only (the golden-fixture generator loads it by path).
"""
from __future__ import annotations

import math

import torch


def make_clip(clip_idx: int, num_frames: int, image_size: int, n_cat: int, n_obj: int, parts=None):
    """Returns {"images": [T, 3, H, W] f32, "masks": [T, n_cat, H, W] bool}.

    `parts` (optional): component counts of categories 0..len(parts)-1.  A category with k > 1
    components holds k smaller discs side by side in its cell (radius cell/(3k+1), spacing
    cell/k: gaps wider than the 5x5 opening), so the frame-0 connected-component split
    (masks.py:13-50) turns it into k tracked objects that the category merge (masks.py:53-213)
    has to recombine."""
    H = W = image_size
    g = torch.Generator().manual_seed(int(clip_idx))
    images = torch.randn(num_frames, 3, H, W, generator=g, dtype=torch.float32)
    grid = int(math.ceil(math.sqrt(n_cat)))
    cell = H // grid
    r = cell / 4.0
    ys = torch.arange(H, dtype=torch.float32).view(H, 1)
    xs = torch.arange(W, dtype=torch.float32).view(1, W)
    masks = torch.zeros(num_frames, n_cat, H, W, dtype=torch.bool)
    parts = list(parts or [])
    for t in range(num_frames):
        for c in range(min(n_obj, n_cat)):
            cx = (c % grid + 0.5) * cell + t
            cy = (c // grid + 0.5) * cell + t
            k = parts[c] if c < len(parts) else 1
            if k <= 1:
                masks[t, c] = (xs - cx) ** 2 + (ys - cy) ** 2 <= r * r
                continue
            rk = cell / (3.0 * k + 1.0)
            for j in range(k):
                jx = cx + (j - (k - 1) / 2.0) * (cell / k)
                masks[t, c] |= (xs - jx) ** 2 + (ys - cy) ** 2 <= rk * rk
    return {"images": images, "masks": masks}


def sam2_collate_fn(batch_list):
    """[{"images": [T,3,H,W], "masks": [T,N,H,W]}] -> BatchedVideoDatapoint (B must be 1)."""
    from .data_utils import BatchedVideoDatapoint, BatchedVideoMetaData

    images = torch.stack([s["images"] for s in batch_list]).permute(1, 0, 2, 3, 4)
    T, B, C, H, W = images.shape
    assert B == 1, f"Only batch_size=1 is supported in the simplified pipeline, got B={B}"
    masks = torch.stack([s["masks"] for s in batch_list]).permute(1, 0, 2, 3, 4)
    N = masks.shape[2]
    t_idx = torch.arange(T, dtype=torch.int32).view(T, 1).expand(T, N)
    obj_to_frame_idx = torch.stack([t_idx, torch.zeros_like(t_idx)], dim=-1).contiguous()
    n_idx = torch.arange(N, dtype=torch.long).view(1, N).expand(T, N)
    objects_identifier = torch.stack(
        [torch.zeros_like(n_idx), n_idx, torch.arange(T, dtype=torch.long).view(T, 1).expand(T, N)], dim=-1
    ).contiguous()
    frame_orig_size = torch.full((T, N, 2), fill_value=H, dtype=torch.long)
    frame_orig_size[..., 1] = W
    masks = masks.reshape(T, B * N, H, W)
    meta = BatchedVideoMetaData(unique_objects_identifier=objects_identifier, frame_orig_size=frame_orig_size)
    return BatchedVideoDatapoint(img_batch=images, obj_to_frame_idx=obj_to_frame_idx, masks=masks.bool(),
                                 metadata=meta, dict_key="video_batch", batch_size=[T])


def synthetic_batch(clip_idx: int, num_frames: int, image_size: int, n_cat: int, n_obj: int, parts=None):
    return sam2_collate_fn([make_clip(clip_idx, num_frames, image_size, n_cat, n_obj, parts)])


class SyntheticClipDataset:
    """Map-style dataset of deterministic synthetic clips (clip index = offset + i), the stand-in
    for the reference's COCODataset (dataset.py:305-343) when no annotation files are present.
    Items are {"images", "masks"} dicts, collated by sam2_collate_fn."""

    def __init__(self, num_clips: int, num_frames: int, image_size: int, n_cat: int, n_obj: int, offset: int = 0,
                 parts=None):
        self.num_clips, self.num_frames, self.image_size = int(num_clips), int(num_frames), int(image_size)
        self.n_cat, self.n_obj, self.offset, self.parts = int(n_cat), int(n_obj), int(offset), parts

    def __len__(self):
        return self.num_clips

    def __getitem__(self, i):
        if not 0 <= i < self.num_clips:
            raise IndexError(i)
        return make_clip(self.offset + i, self.num_frames, self.image_size, self.n_cat, self.n_obj, self.parts)
