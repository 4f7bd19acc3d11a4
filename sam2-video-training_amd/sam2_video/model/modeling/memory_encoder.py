"""MemoryEncoder (reference memory_encoder.py:17-181), NHWC, forward-only.

The encoded memory is detached before it enters the memory bank
(sam2model.py:340-358), so no gradient ever reaches this module: it runs
without an autograd tape.  Mask down-sampler: 4 x (im2col 3x3/2 + GEMM ->
LayerNorm2d -> GELU) then a 1x1 GEMM; pix_feat_proj is evaluated once per
frame and broadcast over objects; CXBlock: depthwise 7x7 kernel -> LN ->
pwconv1 GEMM (GELU) -> pwconv2 GEMM with the layer-scale gamma and the residual
fused in the epilogue; out_proj GEMM to mem_dim.
"""
from __future__ import annotations

import copy
import math

import torch
from torch import nn

from ...kernels import ops
from .layers import Conv2d, Identity, LayerNorm2d, Linear


def _lin(x, mod, act=None, residual=None, cscale=None):
    return ops.linear(x, mod.compute_weight(), mod.bias.detach(), act=act, residual=residual, cscale=cscale)


def fused_add_enabled():
    """S2H_MEMENC_ADD=0: the pixel-feature add as its own broadcast-add launch (A/B)"""
    import os
    return os.environ.get("S2H_MEMENC_ADD", "1") != "0"


class MaskDownSampler(nn.Module):
    def __init__(self, embed_dim=256, kernel_size=4, stride=4, padding=0, total_stride=16, activation=None):
        super().__init__()
        num_layers = int(math.log2(total_stride) // math.log2(stride))
        assert stride ** num_layers == total_stride
        self.k, self.s, self.p = kernel_size, stride, padding
        layers = []
        cin, cout = 1, 1
        for _ in range(num_layers):
            cout = cin * stride ** 2
            layers += [Conv2d(cin, cout, kernel_size, stride, padding), LayerNorm2d(cout), Identity()]
            cin = cout
        layers.append(Conv2d(cout, embed_dim, 1))
        self.encoder = nn.Sequential(*layers)
        self.num_layers = num_layers

    FUSED = {(1, 4), (4, 16), (16, 64)}  # (cin, cout) of the s2h_mask_down_stage kernel

    def _fused(self, conv):
        return (self.k, self.s, self.p) == (3, 2, 1) and (conv.in_ch, conv.out_ch) in self.FUSED

    def forward(self, x=None, logits=None, scale=1.0, shift=0.0, dtype=None, add=None):
        """x [O, H, W, 1] compute dtype, or `logits` [O, H, W] fp32 with the memory-encoder
        input transform sigmoid(logits) * scale + shift fused into the first stage
        -> [O, H/16, W/16, embed_dim]; add [H/16 * W/16, embed_dim] (shared by the objects): added to
        every object's output in the final projection's epilogue"""
        for i in range(self.num_layers):
            conv, ln = self.encoder[3 * i], self.encoder[3 * i + 1]
            if self._fused(conv):
                x = ops.mask_down_stage(x, conv.weight.detach(), conv.bias.detach(), ln.weight.detach(),
                                        ln.bias.detach(), ln.eps, logits=logits, scale=scale, shift=shift,
                                        dtype=dtype)
                logits = None
                continue
            if logits is not None:
                x = ops.act_fwd(logits, "sigmoid", scale=scale, shift=shift)
                x = (ops.cast(x, dtype) if dtype != torch.float32 else x).unsqueeze(-1)
                logits = None
            O = x.shape[0]
            col, Ho, Wo = ops.im2col(x, self.k, self.k, self.s, self.p)
            y = _lin(col, conv).view(O, Ho, Wo, -1)
            y, _, _ = ops.layernorm_fwd(y, ln.weight.detach(), ln.bias.detach(), ln.eps)
            x = ops.act_fwd(y, "gelu")
        proj = self.encoder[3 * self.num_layers]
        if add is None or not fused_add_enabled():
            y = _lin(x, proj)
            return y if add is None else ops.add_bcast(y, add)
        # one batched GEMM (batch = objects) whose residual has batch stride 0: the shared pixel
        # features added in the epilogue (memory_encoder.py:174-175: pix_feat_proj(pix_feat) + masks)
        O, Ho, Wo, K = x.shape
        w = proj.compute_weight()
        N = w.shape[0]
        assert tuple(add.shape) == (Ho * Wo, N) and add.is_contiguous() and x.is_contiguous()
        out = torch.empty(O, Ho, Wo, N, device=x.device, dtype=x.dtype)
        ops.gemm(x.view(O * Ho * Wo, K), w, out.view(-1, N), M=Ho * Wo, N=N, K=K, lda_m=K, lda_k=1, ldb_k=1,
                 ldb_n=K, ldc=N, batch=O, sA=Ho * Wo * K, sB=0, sC=Ho * Wo * N, bias=proj.bias.detach(),
                 residual=add, ldr=N, sR=0)
        return out


class CXBlock(nn.Module):
    def __init__(self, dim, kernel_size=7, padding=3, drop_path=0.0, layer_scale_init_value=1e-6, use_dwconv=True):
        super().__init__()
        assert use_dwconv
        self.pad = padding
        self.dwconv = Conv2d(dim, dim, kernel_size, 1, padding, groups=dim)
        self.norm = LayerNorm2d(dim, eps=1e-6)
        self.pwconv1 = Linear(dim, 4 * dim)
        self.pwconv2 = Linear(4 * dim, dim)
        self.gamma = nn.Parameter(layer_scale_init_value * torch.ones(dim)) if layer_scale_init_value > 0 else None

    def forward(self, x):
        y = ops.dwconv(x, self.dwconv.weight.detach(), self.dwconv.bias.detach(), self.pad)
        y, _, _ = ops.layernorm_fwd(y, self.norm.weight.detach(), self.norm.bias.detach(), self.norm.eps)
        h = _lin(y, self.pwconv1, act="gelu")
        return _lin(h, self.pwconv2, residual=x, cscale=self.gamma.detach() if self.gamma is not None else None)


class Fuser(nn.Module):
    def __init__(self, layer, num_layers, dim=None, input_projection=False):
        super().__init__()
        assert not input_projection
        self.layers = nn.ModuleList([copy.deepcopy(layer) for _ in range(num_layers)])

    def forward(self, x):
        for layer in self.layers:
            x = layer(x)
        return x


class MemoryEncoder(nn.Module):
    def __init__(self, out_dim, mask_downsampler, fuser, position_encoding, in_dim=256):
        super().__init__()
        self.mask_downsampler = mask_downsampler
        self.pix_feat_proj = Conv2d(in_dim, in_dim, 1)
        self.fuser = fuser
        self.position_encoding = position_encoding
        self.out_proj = Conv2d(in_dim, out_dim, 1)
        self.out_dim = out_dim

    @torch.no_grad()
    def forward(self, pix_feat, masks, h, w, scale=1.0, shift=0.0):
        """pix_feat [h*w, C] raw frame features (shared by objects); masks [O, H, W] fp32 mask
        logits, transformed as sigmoid(masks) * scale + shift inside the first down-sampler stage
        -> (features [O, h, w, out_dim], pos table [h*w, out_dim])"""
        O = masks.shape[0]
        p = _lin(pix_feat.detach(), self.pix_feat_proj)  # [h*w, C]
        x = self.mask_downsampler(logits=masks, scale=scale, shift=shift, dtype=pix_feat.dtype, add=p)  # [O, h, w, C]
        x = self.fuser(x)
        x = _lin(x, self.out_proj)
        pos = self.position_encoding.table(h, w, x.device, x.dtype)
        return x.view(O, h, w, self.out_dim), pos
