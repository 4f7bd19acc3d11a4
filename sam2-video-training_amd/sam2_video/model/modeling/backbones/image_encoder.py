"""ImageEncoder + FpnNeck (reference backbones/image_encoder.py:14-134), NHWC.

Lateral 1x1 convs are GEMMs on the NHWC feature rows; the nearest x2 top-down
path is fused with the lateral add (up2_add kernel); the sine positional
encodings are cached device constants (they depend only on the shape)."""
from __future__ import annotations

from typing import List, Optional

import torch
from torch import nn

from ....kernels import functional as FN
from ..layers import Conv2d


class _LateralConv(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.conv = Conv2d(cin, cout, 1)


class FpnNeck(nn.Module):
    def __init__(self, position_encoding, d_model: int, backbone_channel_list: List[int], kernel_size: int = 1,
                 stride: int = 1, padding: int = 0, fpn_interp_model: str = "bilinear", fuse_type: str = "sum",
                 fpn_top_down_levels: Optional[List[int]] = None):
        super().__init__()
        assert kernel_size == 1 and stride == 1 and padding == 0
        assert fpn_interp_model == "nearest" and fuse_type == "sum", "SAM2.1 neck: nearest top-down, sum fuse"
        self.position_encoding = position_encoding
        self.convs = nn.ModuleList(_LateralConv(dim, d_model) for dim in backbone_channel_list)
        self.backbone_channel_list = backbone_channel_list
        self.d_model = d_model
        if fpn_top_down_levels is None:
            fpn_top_down_levels = range(len(self.convs))
        self.fpn_top_down_levels = list(fpn_top_down_levels)

    def forward(self, xs):
        n = len(self.convs) - 1
        out = [None] * len(self.convs)
        pos = [None] * len(self.convs)
        prev = None
        for i in range(n, -1, -1):
            lat = self.convs[n - i].conv(xs[i])
            if i in self.fpn_top_down_levels and prev is not None:
                prev = FN.up2_add(lat, prev)
            else:
                prev = lat
            out[i] = prev
            pos[i] = self.position_encoding.table(prev.shape[1], prev.shape[2], prev.device, prev.dtype)
        return out, pos


class ImageEncoder(nn.Module):
    def __init__(self, trunk, neck, scalp: int = 0):
        super().__init__()
        self.trunk = trunk
        self.neck = neck
        self.scalp = scalp
        assert self.trunk.channel_list == self.neck.backbone_channel_list

    def forward(self, sample_nhwc):
        xs = self.trunk(sample_nhwc)
        # the neck reads aliases of the stage outputs: autograd nodes of their own, so a backward
        # from the backbone outputs can stop at the neck's inputs (the staged backbone backward,
        # SAM2Model.backbone_backward_segments); no data is copied
        xs = [x.view_as(x) for x in xs] if torch.is_grad_enabled() else xs
        self.last_neck_inputs = xs if torch.is_grad_enabled() else []
        features, pos = self.neck(xs)
        if self.scalp > 0:
            features, pos = features[: -self.scalp], pos[: -self.scalp]
        return {"vision_features": features[-1], "vision_pos_enc": pos, "backbone_fpn": features}
