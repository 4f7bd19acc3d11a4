"""Positional encodings.  All of them are constants of the shapes (no parameters
feed them): they are evaluated once on the host with the reference formulas and
cached on the device, like RoPE tables, so the step never recomputes them.

  PositionEmbeddingSine       position_encoding.py:16-130
  PositionEmbeddingRandom     position_encoding.py:133-176 (gaussian buffer kept)
  axial RoPE cos/sin tables   position_encoding.py:186-239
"""
from __future__ import annotations

import math
from typing import Dict, Tuple

import numpy as np
import torch
from torch import nn

_CACHE: Dict[Tuple, torch.Tensor] = {}


def _cached(key, fn):
    t = _CACHE.get(key)
    if t is None:
        t = fn()
        _CACHE[key] = t
    return t


def sine_pe_hwc(H, W, num_pos_feats, temperature=10000, scale=2 * math.pi):
    """[H*W, num_pos_feats] fp32 (CPU) -- PositionEmbeddingSine._pe, normalize=True, NHWC rows."""
    npf = num_pos_feats // 2
    y_embed = torch.arange(1, H + 1, dtype=torch.float32).view(-1, 1).repeat(1, W)
    x_embed = torch.arange(1, W + 1, dtype=torch.float32).view(1, -1).repeat(H, 1)
    eps = 1e-6
    y_embed = y_embed / (y_embed[-1:, :] + eps) * scale
    x_embed = x_embed / (x_embed[:, -1:] + eps) * scale
    dim_t = torch.arange(npf, dtype=torch.float32)
    dim_t = temperature ** (2 * (dim_t // 2) / npf)
    pos_x = x_embed[:, :, None] / dim_t
    pos_y = y_embed[:, :, None] / dim_t
    pos_x = torch.stack((pos_x[:, :, 0::2].sin(), pos_x[:, :, 1::2].cos()), dim=3).flatten(2)
    pos_y = torch.stack((pos_y[:, :, 0::2].sin(), pos_y[:, :, 1::2].cos()), dim=3).flatten(2)
    return torch.cat((pos_y, pos_x), dim=2).reshape(H * W, num_pos_feats)


class PositionEmbeddingSine(nn.Module):
    def __init__(self, num_pos_feats, temperature: int = 10000, normalize: bool = True, scale=None, **kw):
        super().__init__()
        assert num_pos_feats % 2 == 0 and normalize
        self.num_pos_feats = num_pos_feats
        self.temperature = temperature
        self.scale = 2 * math.pi if scale is None else scale

    def table(self, H, W, device, dtype):
        """[H*W, C] device constant"""
        key = ("sine", self.num_pos_feats, self.temperature, self.scale, H, W, str(device), dtype)
        return _cached(key, lambda: sine_pe_hwc(H, W, self.num_pos_feats, self.temperature, self.scale)
                       .to(device=device, dtype=dtype).contiguous())


def pe_random_np(coords, gauss):
    """_pe_encoding (position_encoding.py:147-154) on the host; coords [..., 2] in [0, 1]"""
    c = 2 * coords - 1
    c = c @ gauss
    c = 2 * np.pi * c
    return torch.cat([torch.sin(c), torch.cos(c)], dim=-1)


class PositionEmbeddingRandom(nn.Module):
    def __init__(self, num_pos_feats: int = 64, scale=None):
        super().__init__()
        if scale is None or scale <= 0.0:
            scale = 1.0
        self.register_buffer("positional_encoding_gaussian_matrix", scale * torch.randn((2, num_pos_feats)))

    def _gauss_cpu(self):
        """host copy of the (never-trained) gaussian matrix, refreshed only when the buffer is
        replaced or written: the dense-PE lookup runs inside the captured step, where a
        device->host copy is not allowed"""
        b = self.positional_encoding_gaussian_matrix
        key = (b.data_ptr(), b._version, str(b.device))
        if getattr(self, "_gauss_key", None) != key:
            self._gauss_host = b.detach().float().cpu()
            self._gauss_key = key
        return self._gauss_host

    def dense_table(self, h, w, device, dtype):
        """get_dense_pe (prompt_encoder.py:68-77) as [h*w, C] rows (NHWC)"""
        g = self._gauss_cpu()
        key = ("dense", h, w, str(device), dtype, float(g.sum()), float(g.abs().sum()))

        def make():
            grid = torch.ones((h, w), dtype=torch.float32)
            y = (grid.cumsum(0) - 0.5) / h
            x = (grid.cumsum(1) - 0.5) / w
            pe = pe_random_np(torch.stack([x, y], dim=-1), g)
            return pe.reshape(h * w, -1).to(device=device, dtype=dtype).contiguous()

        return _cached(key, make)

    def points(self, coords, image_size):
        """forward_with_coords (position_encoding.py:169-176) on host coords [B, N, 2] -> [B, N, C] fp32"""
        c = coords.detach().float().cpu().clone()
        c[:, :, 0] = c[:, :, 0] / image_size[1]
        c[:, :, 1] = c[:, :, 1] / image_size[0]
        return pe_random_np(c, self._gauss_cpu())


def axial_rope_table(dim, end_x, end_y, theta, device):
    """compute_axial_cis (position_encoding.py:192-201) as (cos, sin) [end_x*end_y, dim/2] fp32"""
    key = ("rope", dim, end_x, end_y, theta, str(device))

    def make():
        freqs_x = 1.0 / (theta ** (torch.arange(0, dim, 4)[: (dim // 4)].float() / dim))
        freqs_y = 1.0 / (theta ** (torch.arange(0, dim, 4)[: (dim // 4)].float() / dim))
        t = torch.arange(end_x * end_y, dtype=torch.float32)
        t_x = (t % end_x).float()
        t_y = torch.div(t, end_x, rounding_mode="floor").float()
        ang = torch.cat([torch.outer(t_x, freqs_x), torch.outer(t_y, freqs_y)], dim=-1)
        cis = torch.polar(torch.ones_like(ang), ang)
        return (cis.real.float().contiguous().to(device), cis.imag.float().contiguous().to(device))

    return _cached(key, make)


def get_1d_sine_pe(pos_inds, dim, temperature=10000):
    """sam2_utils.py:64-74 (host)"""
    pe_dim = dim // 2
    dim_t = torch.arange(pe_dim, dtype=torch.float32)
    dim_t = temperature ** (2 * (dim_t // 2) / pe_dim)
    pos_embed = pos_inds.unsqueeze(-1) / dim_t
    return torch.cat([pos_embed.sin(), pos_embed.cos()], dim=-1)
