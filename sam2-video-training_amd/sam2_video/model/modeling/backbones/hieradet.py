"""Hiera trunk (reference: sam2_video/model/modeling/backbones/hieradet.py, upstream
sam2.modeling.backbones.hieradet), NHWC on the device.

Same constructor signature / parameter names as the reference (hieradet.py:169-262)
so SAM2.1 checkpoints load.  Per block: LayerNorm kernel -> (proj + 2x2 max-pool
shortcut) -> window partition (zero pad; windows that need padding partition the qkv
projection of the real tokens with bias rows instead) -> fused qkv GEMM -> (q max-pool read
in place from the qkv tensor) -> flash attention over [windows, L, heads, d] ->
proj GEMM -> unpartition -> residual-add fused into norm2 -> MLP GEMMs (GELU in
the epilogue, residual in the second epilogue).
"""
from __future__ import annotations

import os
from typing import List, Tuple

import torch
from torch import nn

from ....kernels import functional as FN
from ....kernels import ops
from ....kernels.functional_sam import hiera_pos_embed
from ..layers import MLP, Conv2d, LayerNorm, Linear


def _stage_windows():
    """S2H_HIERA_WIN_STAGE=0: every windowed block partitions its normed input and unpartitions its
    attention output, as the reference does (hieradet.py:146,161), instead of the stage-level window order"""
    return os.environ.get("S2H_HIERA_WIN_STAGE", "1") == "1"


def _pad_after_qkv():
    """S2H_HIERA_PAD_QKV=0: padded windows partition the normed input (zero rows) before the qkv
    projection, as the reference does, instead of the projection's output (bias rows)"""
    return os.environ.get("S2H_HIERA_PAD_QKV", "1") == "1"


class MultiScaleAttention(nn.Module):
    """hieradet.py:39-81"""

    def __init__(self, dim: int, dim_out: int, num_heads: int, q_pool: bool = False):
        super().__init__()
        self.dim, self.dim_out, self.num_heads, self.q_pool = dim, dim_out, num_heads, q_pool
        self.qkv = Linear(dim, dim_out * 3)
        self.proj = Linear(dim_out, dim_out)

    def forward(self, x):
        B, H, W, _ = x.shape
        d, nh = self.dim_out, self.num_heads
        qkv = self.qkv(x)  # [B, H, W, 3d]
        qkv5 = qkv.view(B, H * W, 3, nh, d // nh)
        if self.q_pool:  # q pooled straight out of the fused qkv; one dqkv in the backward
            o = FN.pooled_qkv_attention(qkv, nh)
            H, W = H // 2, W // 2
        else:
            o = FN.qkv_attention(qkv5)  # one packed dqkv in the backward
        return self.proj(o.reshape(B, H, W, d))


class MultiScaleBlock(nn.Module):
    """hieradet.py:84-166"""

    def __init__(self, dim, dim_out, num_heads, mlp_ratio=4.0, drop_path=0.0, norm_layer="LayerNorm",
                 q_stride=None, act_layer=None, window_size=0):
        super().__init__()
        self.dim, self.dim_out = dim, dim_out
        self.norm1 = LayerNorm(dim, eps=1e-6)
        self.window_size = window_size
        self.q_stride = q_stride
        self.attn = MultiScaleAttention(dim, dim_out, num_heads=num_heads, q_pool=bool(q_stride))
        self.norm2 = LayerNorm(dim_out, eps=1e-6)
        self.mlp = MLP(dim_out, int(dim_out * mlp_ratio), dim_out, num_layers=2, activation="gelu")
        if dim != dim_out:
            self.proj = Linear(dim, dim_out)

    def forward(self, x, xn=None, next_norm=None, windowed=False):
        """x: residual stream [B, H, W, C]; xn = norm1(x) when the previous block already produced
        it (fused with its residual add).  With next_norm, returns (x', next_norm(x')) from one
        fused add + LayerNorm so the stream has a single autograd consumer; else x'.
        windowed: x is already in window order, [B * windows, ws, ws, C] (Hiera.forward keeps a
        stage whose blocks all use whole windows of one grid in that order): every op of the block
        but the attention is per token and the 2x2 q-pool stays inside a window, so the block runs
        on the windows as they are, with no partition / unpartition of its own"""
        B = x.shape[0]
        if xn is None:
            xn = self.norm1(x)
        shortcut = x
        if self.dim != self.dim_out:
            shortcut = self.proj(xn)
            if self.q_stride:
                shortcut = FN.maxpool2(shortcut)
        ws = self.window_size
        H, W = xn.shape[1:3]
        if windowed:
            y = self.attn(xn)
        elif ws > 0 and not self.q_stride and (H % ws or W % ws) and _pad_after_qkv():
            # windows that need padding (stage 3: 32 -> 42, stage 4: 16 -> 21 at 512^2): the qkv
            # projection of a zero-padded row is its bias, so project the real tokens only, partition
            # the projection with bias rows, and project back after unpartition -- the qkv and proj
            # GEMMs (and their backward) run on H*W instead of the padded rows (0.58x at 512^2)
            a = self.attn
            qkvw = FN.window_pad(a.qkv(xn), ws, a.qkv)
            nwin, d, nh = qkvw.shape[0], a.dim_out, a.num_heads
            o = FN.qkv_attention(qkvw.view(nwin, ws * ws, 3, nh, d // nh))
            y = a.proj(FN.window_unpartition(o.reshape(nwin, ws, ws, d), ws, B, H, W))
        else:
            xw = FN.window_partition(xn, ws) if ws > 0 else xn
            y = self.attn(xw)
            if self.q_stride:
                ws = ws // self.q_stride[0]
                H, W = shortcut.shape[1:3]
            if self.window_size > 0:
                y = FN.window_unpartition(y, ws, B, H, W)
        h, x = FN.add_layer_norm(shortcut, y, self.norm2, self.norm2.eps)
        fc1, fc2 = self.mlp.layers[0], self.mlp.layers[1]
        if next_norm is None:
            return FN.mlp2(h, fc1, fc2, "gelu", residual=x)
        t, x = FN.add_layer_norm(x, FN.mlp2(h, fc1, fc2, "gelu"), next_norm, next_norm.eps)
        return x, t


class PatchEmbed(nn.Module):
    """backbones/utils.py:63-93 -- conv 7x7/4 as im2col + GEMM"""

    def __init__(self, kernel_size=(7, 7), stride=(4, 4), padding=(3, 3), in_chans=3, embed_dim=768):
        super().__init__()
        self.k, self.s, self.p = kernel_size[0], stride[0], padding[0]
        self.proj = Conv2d(in_chans, embed_dim, self.k, self.s, self.p)

    def forward(self, x_nhwc):
        T = x_nhwc.shape[0]
        col, Ho, Wo = ops.im2col(x_nhwc, self.k, self.k, self.s, self.p, pad8=True)
        return self.proj(col).view(T, Ho, Wo, -1)


class Hiera(nn.Module):
    """hieradet.py:169-299"""

    def __init__(self, embed_dim: int = 96, num_heads: int = 1, drop_path_rate: float = 0.0, q_pool: int = 3,
                 q_stride: Tuple[int, int] = (2, 2), stages=(2, 3, 16, 3), dim_mul: float = 2.0,
                 head_mul: float = 2.0, window_pos_embed_bkg_spatial_size=(14, 14), window_spec=(8, 4, 14, 7),
                 global_att_blocks=(12, 16, 20), weights_path=None, return_interm_layers=True):
        super().__init__()
        assert len(stages) == len(window_spec)
        self.window_spec = window_spec
        depth = sum(stages)
        self.q_stride = tuple(q_stride)
        self.stage_ends = [sum(stages[:i]) - 1 for i in range(1, len(stages) + 1)]
        self.q_pool_blocks = [x + 1 for x in self.stage_ends[:-1]][:q_pool]
        self.return_interm_layers = return_interm_layers
        self.patch_embed = PatchEmbed(embed_dim=embed_dim)
        self.global_att_blocks = global_att_blocks
        self.window_pos_embed_bkg_spatial_size = window_pos_embed_bkg_spatial_size
        self.pos_embed = nn.Parameter(torch.zeros(1, embed_dim, *window_pos_embed_bkg_spatial_size))
        self.pos_embed_window = nn.Parameter(torch.zeros(1, embed_dim, window_spec[0], window_spec[0]))
        cur_stage = 1
        self.blocks = nn.ModuleList()
        for i in range(depth):
            dim_out = embed_dim
            window_size = self.window_spec[cur_stage - 1]
            if self.global_att_blocks is not None:
                window_size = 0 if i in self.global_att_blocks else window_size
            if i - 1 in self.stage_ends:
                dim_out = int(embed_dim * dim_mul)
                num_heads = int(num_heads * head_mul)
                cur_stage += 1
            self.blocks.append(MultiScaleBlock(dim=embed_dim, dim_out=dim_out, num_heads=num_heads,
                                               q_stride=self.q_stride if i in self.q_pool_blocks else None,
                                               window_size=window_size))
            embed_dim = dim_out
        self.channel_list = ([self.blocks[i].dim_out for i in self.stage_ends[::-1]] if return_interm_layers
                             else [self.blocks[-1].dim_out])

    def window_stages(self, H, W):
        """{first block: (last block, window size at the stage's input)} of the stages whose blocks
        all attend within whole (unpadded) windows of one grid -- the q-pool block that opens a stage
        halves the window with the image, so its output windows are the next blocks' (at 512^2:
        stage 1, 8x8 windows of 128^2, and stage 2, 8x8 -> 4x4 windows of 128^2 -> 64^2).  Such a
        stage runs in window order between one partition at its start and one unpartition at its end
        instead of both around every block's attention (hieradet.py:146,161)."""
        runs = {}
        if not _stage_windows():
            return runs
        b0 = 0
        for b1 in self.stage_ends:
            h, w, ok, ws_cur = H, W, True, None
            for i in range(b0, b1 + 1):
                blk = self.blocks[i]
                ws = blk.window_size
                if ws <= 0 or h % ws or w % ws or (ws_cur is not None and ws != ws_cur):
                    ok = False
                if blk.q_stride:
                    ok = ok and ws % blk.q_stride[0] == 0 and tuple(blk.q_stride) == (2, 2)
                    h, w, ws_cur = h // 2, w // 2, ws // 2
                else:
                    ws_cur = ws
            if ok:
                runs[b0] = (b1, self.blocks[b0].window_size)
            H, W = h, w
            b0 = b1 + 1
        return runs

    def forward(self, x_nhwc) -> List[torch.Tensor]:
        """x: [T, H, W, 3] compute dtype -> stage outputs NHWC (high -> low resolution)"""
        x = self.patch_embed(x_nhwc)
        pe = hiera_pos_embed(self.pos_embed, self.pos_embed_window, x.shape[1], x.shape[2], x.dtype)
        x = FN.add_bcast(x, pe)
        outputs = []
        t = None
        runs = self.window_stages(x.shape[1], x.shape[2])
        run_end, img = -1, None  # last block of the window-ordered stage, its output's (B, H, W, ws)
        for i, blk in enumerate(self.blocks):
            is_out = (i == self.stage_ends[-1]) or (i in self.stage_ends and self.return_interm_layers)
            if i in runs:
                run_end, ws = runs[i]
                B, H, W = x.shape[:3]
                for j in range(i, run_end + 1):
                    if self.blocks[j].q_stride:
                        H, W, ws = H // 2, W // 2, ws // 2
                img = (B, H, W, ws)
                x = FN.window_partition(x, runs[i][1])  # (t is None: see below)
            windowed = i <= run_end
            if is_out or i + 1 == len(self.blocks) or i == run_end or i + 1 in runs:
                x, t = blk(x, t, windowed=windowed), None
            else:
                x, t = blk(x, t, next_norm=self.blocks[i + 1].norm1, windowed=windowed)
            if i == run_end:
                x = FN.window_unpartition(x, img[3], *img[:3])
            if is_out:
                outputs.append(x)
        # the stage outputs: the cut points of the staged backbone backward
        # (SAM2Model.backbone_backward_segments)
        self.last_outputs = outputs if torch.is_grad_enabled() else []
        return outputs
