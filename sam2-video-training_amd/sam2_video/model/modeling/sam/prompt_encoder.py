"""PromptEncoder (reference sam/prompt_encoder.py:17-202).

Point/box clicks are host-side data (generated on the host from the frame-0
masks, as in the reference); their random-Fourier encodings are evaluated on the
host with the module's gaussian buffer, and the learned label embeddings are
added on the device by the point_embed kernel (whose backward accumulates the
label-embedding gradients).  The dense embedding without a mask prompt is the
`no_mask_embed` broadcast, folded into the decoder's image-embedding add.
"""
from __future__ import annotations

import torch
from torch import nn

from ....kernels import ops
from ....kernels.functional_sam import point_embed
from ..layers import Conv2d, Embedding, Identity, LayerNorm2d
from ..position_encoding import PositionEmbeddingRandom


class PromptEncoder(nn.Module):
    def __init__(self, embed_dim, image_embedding_size, input_image_size, mask_in_chans, activation=None):
        super().__init__()
        self.embed_dim = embed_dim
        self.input_image_size = tuple(input_image_size)
        self.image_embedding_size = tuple(image_embedding_size)
        self.pe_layer = PositionEmbeddingRandom(embed_dim // 2)
        self.num_point_embeddings = 4
        self.point_embeddings = nn.ModuleList([Embedding(1, embed_dim) for _ in range(4)])
        self.not_a_point_embed = Embedding(1, embed_dim)
        self.mask_input_size = (4 * image_embedding_size[0], 4 * image_embedding_size[1])
        self.mask_downscaling = nn.Sequential(
            Conv2d(1, mask_in_chans // 4, 2, 2), LayerNorm2d(mask_in_chans // 4), Identity(),
            Conv2d(mask_in_chans // 4, mask_in_chans, 2, 2), LayerNorm2d(mask_in_chans), Identity(),
            Conv2d(mask_in_chans, embed_dim, 1))
        self.no_mask_embed = Embedding(1, embed_dim)

    def dense_pe_table(self, device, dtype):
        """get_dense_pe as [h*w, C] rows"""
        h, w = self.image_embedding_size
        return self.pe_layer.dense_table(h, w, device, dtype)

    def host_points(self, coords, labels, pad=True):
        """_embed_points' coordinate part (prompt_encoder.py:79-95) on the host:
        returns (pe [B, N(+1), C] fp32, labels [B, N(+1)] int32) with the padding click."""
        coords = coords.detach().float().cpu() + 0.5
        labels = labels.detach().cpu().to(torch.int32)
        if pad:
            coords = torch.cat([coords, torch.zeros(coords.shape[0], 1, 2)], dim=1)
            labels = torch.cat([labels, -torch.ones(labels.shape[0], 1, dtype=torch.int32)], dim=1)
        pe = self.pe_layer.points(coords, self.input_image_size)
        return pe, labels

    def sparse(self, pe_dev, labels_dev, dtype):
        """label embeddings added on the device -> [B, N, C] (differentiable in the embeddings)"""
        return point_embed(pe_dev, labels_dev, dtype, self.not_a_point_embed, self.point_embeddings)

    @torch.no_grad()
    def dense_from_mask(self, masks, dtype):
        """_embed_masks (prompt_encoder.py:153-158) on NHWC masks [B, 4h, 4w, 1]: conv2x2/2 -> LN2d ->
        GELU -> conv2x2/2 -> LN2d -> GELU -> conv1x1, as im2col GEMMs + row norms; returns the dense
        embedding [B, h*w, C].  Forward only (the mask-prompt frame takes no gradient)."""
        from ....kernels.functional import _compute_weight
        x = ops.cast(masks.contiguous(), dtype) if masks.dtype != dtype else masks
        B = x.shape[0]
        c0, n1, _, c3, n4, _, c6 = self.mask_downscaling
        for conv, norm in ((c0, n1), (c3, n4)):
            col, Ho, Wo = ops.im2col(x.contiguous(), 2, 2, 2, 0)
            y = ops.linear(col, _compute_weight(conv), conv.bias.detach())
            y, _, _ = ops.layernorm_fwd(y, norm.weight.detach(), norm.bias.detach(), norm.eps)
            x = ops.act_fwd(y, "gelu").view(B, Ho, Wo, -1)
        y = ops.linear(x.reshape(-1, x.shape[-1]), _compute_weight(c6), c6.bias.detach())
        return y.view(B, -1, self.embed_dim)
