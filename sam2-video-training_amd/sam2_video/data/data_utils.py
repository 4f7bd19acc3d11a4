"""Batch container of the training step.

Mirrors `BatchedVideoDatapoint` / `BatchedVideoMetaData`
(reference: sam2_video/data/data_utils.py:21-86) with the same attribute names
and properties.  The reference builds them with tensordict's @tensorclass; this
build keeps a plain dataclass (tensordict is not a dependency) that supports the
operations the hot path uses: `.to(device)`, `.pin_memory()`, `num_frames`,
`num_videos`, `flat_obj_to_img_idx`, `flat_img_batch`.
"""
from __future__ import annotations

from dataclasses import dataclass, field, fields
from typing import List

import torch


def _map(obj, fn):
    kw = {}
    for f in fields(obj):
        v = getattr(obj, f.name)
        if isinstance(v, torch.Tensor):
            v = fn(v)
        elif hasattr(v, "__dataclass_fields__"):
            v = _map(v, fn)
        kw[f.name] = v
    return type(obj)(**kw)


@dataclass
class BatchedVideoMetaData:
    """unique_objects_identifier [T, N, 3] (video_id, obj_id, frame_id); frame_orig_size [T, N, 2]."""
    unique_objects_identifier: torch.Tensor
    frame_orig_size: torch.Tensor


@dataclass
class BatchedVideoDatapoint:
    """img_batch [T, B, C, H, W] f32; obj_to_frame_idx [T, O, 2] int32; masks [T, O, H, W] bool."""
    img_batch: torch.Tensor
    obj_to_frame_idx: torch.Tensor
    masks: torch.Tensor
    metadata: BatchedVideoMetaData
    dict_key: str
    batch_size: List[int] = field(default_factory=list)

    def __post_init__(self):
        if not self.batch_size:
            self.batch_size = [int(self.img_batch.shape[0])]

    def to(self, device, non_blocking=False):
        out = _map(self, lambda t: t.to(device, non_blocking=non_blocking))
        # keep the host copy of frame 0's masks: connected components + clicks are host-side
        # work (masks.py:13-50, prompts.py) and can run without a device->host sync
        hm = getattr(self, "host_masks0", None)
        out.host_masks0 = hm if hm is not None else (self.masks[0] if not self.masks.is_cuda else None)
        return out

    def pin_memory(self, device=None):
        return _map(self, lambda t: t.pin_memory())

    @property
    def num_frames(self) -> int:
        return self.batch_size[0]

    @property
    def num_videos(self) -> int:
        return self.img_batch.shape[1]

    @property
    def flat_obj_to_img_idx(self) -> torch.Tensor:
        frame_idx, video_idx = self.obj_to_frame_idx.unbind(dim=-1)
        return video_idx * self.num_frames + frame_idx

    @property
    def flat_img_batch(self) -> torch.Tensor:
        """[(B*T), C, H, W] (reference data_utils.py:80-86)"""
        return self.img_batch.transpose(0, 1).flatten(0, 1)
