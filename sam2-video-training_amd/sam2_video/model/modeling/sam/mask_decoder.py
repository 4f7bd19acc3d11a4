"""MaskDecoder (reference sam/mask_decoder.py:15-245), batch-first NHWC.

Single-mask path (multimask_output=False, mask_decoder.py:151-153): only the
hypernetwork MLP of mask token 0 feeds the returned mask, so only that product
is evaluated (the other three MLPs are in the graph of the reference with zero
gradient; they stay in the optimizer's gradient arena with zero gradients, which
keeps AdamW's weight decay identical).  Upscaling: ConvTranspose2x2 GEMMs with
the scatter + bias + high-res skip add fused, LayerNorm2d as a row norm (NHWC),
GELU kernels, hypernetwork mask as a batched GEMM.
"""
from __future__ import annotations

import torch
from torch import nn

from ....kernels import frametape as _ft
from ....kernels import functional as FN
from ....kernels import ops
from ....kernels.functional_sam import conv_transpose2x2, hyper_mask
from ..layers import MLP, Conv2d, ConvTranspose2x2, Embedding, Identity, LayerNorm2d, Linear


class _DecoderTokens(torch.autograd.Function):
    """cat(obj_score_token, iou_token, mask_tokens) expanded over objects, then the sparse prompts
    (mask_decoder.py:178-195); backward sums the token gradients over objects into the arena."""

    @staticmethod
    def forward(ctx, sparse, dtype, *params):
        O, Ns, C = sparse.shape
        head = torch.cat([p._s2h_compute.reshape(-1, C) for p in params], 0)
        nh = head.shape[0]
        out = torch.empty(O, nh + Ns, C, device=sparse.device, dtype=dtype)
        out[:, :nh].copy_(head.unsqueeze(0).expand(O, -1, -1))
        out[:, nh:].copy_(sparse)
        ctx.params = params
        ctx.nh = nh
        return out

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        C = g.shape[-1]
        r = 0
        for p in ctx.params:
            gp = getattr(p, "_s2h_grad", None) if p.requires_grad else None
            n = p.numel() // C
            if gp is not None:
                for j in range(n):
                    ops.colsum(g[:, r + j], gp.view(-1, C)[j], accumulate=True)
            r += n
        return (g[:, ctx.nh:],) + (None,) * (1 + len(ctx.params))


class MaskDecoder(nn.Module):
    def __init__(self, *, transformer_dim, transformer, num_multimask_outputs=3, activation=None, iou_head_depth=3,
                 iou_head_hidden_dim=256, use_high_res_features=False, iou_prediction_use_sigmoid=False,
                 dynamic_multimask_via_stability=False, dynamic_multimask_stability_delta=0.05,
                 dynamic_multimask_stability_thresh=0.98, pred_obj_scores=False, pred_obj_scores_mlp=False,
                 use_multimask_token_for_obj_ptr=False):
        super().__init__()
        assert use_high_res_features and pred_obj_scores, "SAM2.1 decoder (high-res features, object scores)"
        self.transformer_dim = transformer_dim
        self.transformer = transformer
        self.num_multimask_outputs = num_multimask_outputs
        self.iou_token = Embedding(1, transformer_dim)
        self.num_mask_tokens = num_multimask_outputs + 1
        self.mask_tokens = Embedding(self.num_mask_tokens, transformer_dim)
        self.pred_obj_scores = pred_obj_scores
        self.obj_score_token = Embedding(1, transformer_dim)
        self.use_multimask_token_for_obj_ptr = use_multimask_token_for_obj_ptr
        self.output_upscaling = nn.Sequential(
            ConvTranspose2x2(transformer_dim, transformer_dim // 4), LayerNorm2d(transformer_dim // 4), Identity(),
            ConvTranspose2x2(transformer_dim // 4, transformer_dim // 8), Identity())
        self.use_high_res_features = use_high_res_features
        self.conv_s0 = Conv2d(transformer_dim, transformer_dim // 8, 1)
        self.conv_s1 = Conv2d(transformer_dim, transformer_dim // 4, 1)
        self.output_hypernetworks_mlps = nn.ModuleList(
            [MLP(transformer_dim, transformer_dim, transformer_dim // 8, 3) for _ in range(self.num_mask_tokens)])
        self.iou_prediction_head = MLP(transformer_dim, iou_head_hidden_dim, self.num_mask_tokens, iou_head_depth,
                                       sigmoid_output=iou_prediction_use_sigmoid)
        self.pred_obj_score_head = (MLP(transformer_dim, transformer_dim, 1, 3) if pred_obj_scores_mlp
                                    else Linear(transformer_dim, 1))

    def forward(self, image_embeddings, h, w, image_pe_table, sparse, no_mask_embed, high_res_features, dense=None,
                defer_score=False):
        """image_embeddings [O, h*w, C]; sparse [O, Ns, C]; high_res_features (s0 [1|O, 4h, 4w, C/8],
        s1 [1|O, 2h, 2w, C/4]) -> (low-res mask logits [O, 4h*4w] compute dtype, iou [O, 1],
        mask token 0 [O, C], object score logits [O, 1] f32)"""
        O = image_embeddings.shape[0]
        C = self.transformer_dim
        dt = image_embeddings.dtype
        tparams = (self.obj_score_token.weight, self.iou_token.weight, self.mask_tokens.weight)
        T = _ft.active()
        tokens = (_ft.decoder_tokens(T, sparse, dt, tparams) if T is not None
                  else _DecoderTokens.apply(sparse, dt, *tparams))
        if dense is None:  # no mask prompt: the no_mask_embed broadcast (prompt_encoder.py:196-200)
            src = FN.add_bcast(image_embeddings, no_mask_embed.weight._s2h_compute.view(-1), bparam=no_mask_embed.weight)
        else:  # mask-prompt dense embedding [O, h*w, C]
            src = FN.add(image_embeddings, dense)
        hs, src = self.transformer(src, image_pe_table, tokens)
        iou_token_out, mask_token0 = FN.select_tokens(hs, (1, 2))
        feat_s0, feat_s1 = high_res_features
        dc1, ln1, _, dc2, _ = self.output_upscaling
        u = src.view(O, h, w, C)
        if T is not None and _ft.convt_ln_gelu_ok(u, dc1, feat_s1, ln1):
            # dc1 + feat_s1, LayerNorm2d and GELU in one launch after the GEMM (frametape.convt_ln_gelu)
            u = _ft.convt_ln_gelu(T, u, dc1, feat_s1, ln1)
        else:
            u = conv_transpose2x2(u, dc1, add=feat_s1)
            u = FN.act(ln1(u), "gelu")
        # the hypernetwork MLP of mask token 0 and the IoU head: one launch (FN.mlp_heads)
        hyper0, iou_pred = FN.mlp_heads([(self.output_hypernetworks_mlps[0], mask_token0),
                                         (self.iou_prediction_head, iou_token_out)])
        if T is not None and _ft.convt_tail_ok(u, dc2, feat_s0, hyper0):
            # dc2 + feat_s0, GELU and the mask head in one launch after the GEMM (frametape.convt_tail)
            masks = _ft.convt_tail(T, u, dc2, feat_s0, hyper0)
        else:
            u = conv_transpose2x2(u, dc2, add=feat_s0)
            u = FN.act(u, "gelu")
            masks = hyper_mask(hyper0, u.view(O, -1, C // 8))
        iou0 = FN.cast(FN.select_token(iou_pred.unsqueeze(-1), 0), torch.float32)
        if defer_score:  # the caller runs the object-score head with its other no-grad heads (one launch)
            return masks, iou0, mask_token0, hs[:, 0].detach()
        with torch.no_grad():
            score = self.pred_obj_score_head(hs[:, 0].detach().contiguous())
            score = ops.cast(score, torch.float32) if score.dtype != torch.float32 else score
        return masks, iou0, mask_token0, score
