"""COCO-format video clips (reference sam2_video/data/dataset.py:28-343) without torchvision /
pycocotools (not installed here): same classes, constructor arguments and item layout.

* COCOImageDataset: the COCO JSON's keyframe images (`is_det_keyframe`), categories mapped to
  contiguous indices by sorted id, per-image category masks = OR of the RLE-decoded instance
  masks (data/rle.py), each resized (nearest, short side -> image_size) and center-cropped;
  images resized (bilinear, short side), center-cropped, scaled to [0, 1] and ImageNet
  normalised -- torchvision's Resize(int) / CenterCrop / ToTensor / Normalize semantics.
  Images whose masks are all empty are skipped (next index), as the reference does.
* VideoDataset: fixed-length clips of each video (frames sorted by `order_in_video`), clip
  starts every `stride` frames.
* COCODataset: the two combined; items {"images": [T, 3, S, S], "masks": [T, N, S, S] bool},
  collated by data.synthetic.sam2_collate_fn into BatchedVideoDatapoint.

Host-side work (the reference runs it in DataLoader workers as well).
"""
from __future__ import annotations

import json
from pathlib import Path
from typing import Any, Dict, List, Optional

import numpy as np
import torch
import torch.nn.functional as F

from . import rle as _rle

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def _cfg(config, key, default=None):
    if isinstance(config, dict):
        return config.get(key, default)
    return getattr(config, key, default)


def resized_hw(h: int, w: int, size: int):
    """torchvision Resize(int): the short side becomes `size`, the long side int(size * long / short)"""
    if w <= h:
        return int(size * h / w), size
    return size, int(size * w / h)


def center_crop_box(h: int, w: int, th: int, tw: int):
    """torchvision center_crop offsets (top, left)"""
    return int(round((h - th) / 2.0)), int(round((w - tw) / 2.0))


def load_image(path: str, size: int) -> torch.Tensor:
    """RGB image -> [3, size, size] f32: bilinear resize of the short side (PIL), center crop,
    /255, ImageNet normalisation (dataset.py:103-110)"""
    from PIL import Image
    img = Image.open(path).convert("RGB")
    w, h = img.size
    nh, nw = resized_hw(h, w, size)
    img = img.resize((nw, nh), Image.BILINEAR)
    top, left = center_crop_box(nh, nw, size, size)
    img = img.crop((left, top, left + size, top + size))
    x = torch.from_numpy(np.asarray(img, dtype=np.uint8).copy()).permute(2, 0, 1).float().div_(255.0)
    mean = torch.tensor(IMAGENET_MEAN).view(3, 1, 1)
    std = torch.tensor(IMAGENET_STD).view(3, 1, 1)
    return (x - mean) / std


def resize_mask(m: np.ndarray, size: int) -> torch.Tensor:
    """uint8 mask [H, W] -> bool [size, size]: nearest resize of the short side, center crop
    (dataset.py:166-169)"""
    t = torch.from_numpy(m).float()[None, None]
    h, w = m.shape
    nh, nw = resized_hw(h, w, size)
    t = F.interpolate(t, size=(nh, nw), mode="nearest")[0, 0]
    top, left = center_crop_box(nh, nw, size, size)
    return t[top:top + size, left:left + size] > 0.5


class COCOImageDataset(torch.utils.data.Dataset):
    """dataset.py:28-216"""

    def __init__(self, config: Any, json_path: Optional[str] = None):
        self.config = config
        self.coco_json_path = Path(json_path or _cfg(config, "train_path"))
        self.image_size = int(_cfg(config, "image_size"))
        if not self.coco_json_path.exists():
            raise FileNotFoundError(f"COCO JSON file not found: {self.coco_json_path}")
        with open(self.coco_json_path) as f:
            coco = json.load(f)
        self.images: List[Dict[str, Any]] = [img for img in coco.get("images", []) if img["is_det_keyframe"]]
        self.annotations: List[Dict[str, Any]] = coco.get("annotations", [])
        self.categories: List[Dict[str, Any]] = coco.get("categories", [])
        if not self.categories:
            raise ValueError("COCO JSON must include non-empty 'categories' list for fail-fast semantics")
        sorted_cats = sorted(self.categories, key=lambda c: c.get("id", 0))
        self.catid_to_idx = {c["id"]: i for i, c in enumerate(sorted_cats)}
        n = _cfg(config, "num_categories")
        self.num_categories = int(n) if n is not None else len(sorted_cats)
        self.image_id_to_annotations: Dict[int, List[Dict]] = {}
        for ann in self.annotations:
            self.image_id_to_annotations.setdefault(ann["image_id"], []).append(ann)
        self.video_to_images: Dict[Any, List[Dict]] = {}
        for img in self.images:
            self.video_to_images.setdefault(img.get("video_id", 0), []).append(img)
        for vid in self.video_to_images:
            self.video_to_images[vid].sort(key=lambda x: x.get("order_in_video", 0))
        self.image_id_to_idx = {img["id"]: i for i, img in enumerate(self.images)}
        self.mask_cache: Dict[int, torch.Tensor] = {}

    def _load_gt_masks_for_image(self, image_id: int) -> torch.Tensor:
        """dataset.py:139-179: [num_categories, S, S] bool, instances of a category OR-ed"""
        if image_id in self.mask_cache:
            return self.mask_cache[image_id]
        S = self.image_size
        masks = torch.zeros((self.num_categories, S, S), dtype=torch.bool)
        for ann in self.image_id_to_annotations.get(image_id, []):
            seg, cat_id = ann.get("segmentation"), ann.get("category_id")
            if seg is None or cat_id is None:
                continue
            ci = self.catid_to_idx.get(cat_id)
            if ci is None or ci >= self.num_categories:
                continue
            masks[ci] |= resize_mask(_rle.decode(seg), S)
        self.mask_cache[image_id] = masks
        return masks

    def __len__(self):
        return len(self.images)

    def __getitem__(self, idx):
        """dataset.py:184-216 (an image without any mask pixel is replaced by the next one)"""
        for _ in range(len(self.images)):
            info = self.images[idx]
            masks = self._load_gt_masks_for_image(info["id"])
            if masks.sum() > 0:
                return {"image": load_image(info["path"], self.image_size), "masks": masks}
            idx = (idx + 1) % len(self.images)
        raise RuntimeError("every image of the dataset has empty masks")


class VideoDataset(torch.utils.data.Dataset):
    """dataset.py:219-302"""

    def __init__(self, image_dataset: COCOImageDataset, config: Any):
        self.image_dataset = image_dataset
        self.config = config
        self.video_clip_length = int(_cfg(config, "video_clip_length"))
        self.stride = int(_cfg(config, "stride"))
        self.image_size = int(_cfg(config, "image_size"))
        self.clip_indices: List[Dict[str, Any]] = []
        for vid, images in image_dataset.video_to_images.items():
            start = 0
            while start + self.video_clip_length <= len(images):
                idxs = [image_dataset.image_id_to_idx[images[start + i]["id"]] for i in range(self.video_clip_length)]
                self.clip_indices.append({"video_id": vid, "clip_start": start, "image_indices": idxs})
                start += self.stride

    def __len__(self):
        return len(self.clip_indices)

    def __getitem__(self, idx):
        items = [self.image_dataset[i] for i in self.clip_indices[idx]["image_indices"]]
        return {"images": torch.stack([it["image"] for it in items]),
                "masks": torch.stack([it["masks"] for it in items])}


class COCODataset(torch.utils.data.Dataset):
    """dataset.py:305-343"""

    def __init__(self, config: Any, coco_json_path: Optional[str] = None):
        self.config = config
        image_dataset = COCOImageDataset(config=config, json_path=coco_json_path or _cfg(config, "train_path"))
        self.video_dataset = VideoDataset(image_dataset=image_dataset, config=config)

    def __len__(self):
        return len(self.video_dataset)

    def __getitem__(self, idx):
        return self.video_dataset[idx]

