"""Attention modules (reference sam/transformer.py:19-311), batch-first [B, L, C].

Attention: q/k/v projection GEMMs, flash attention over [B, L, heads, d] views
of the projections (no head transposes), out-projection GEMM with the residual
add fused in its epilogue.  RoPEAttention adds the axial 2-D rotary encoding
(q fully, k on the first Lk - num_k_exclude_rope rows with the table repeated
every Lq rows, i.e. rope_k_repeat) using cached cos/sin tables."""
from __future__ import annotations

import math

import torch
from torch import nn

from ....kernels import frametape as _ft
from ....kernels import functional as FN
from ....kernels import ops
from ..layers import MLP, LayerNorm, Linear
from ..position_encoding import axial_rope_table


class Attention(nn.Module):
    """transformer.py:190-248"""

    def __init__(self, embedding_dim, num_heads, downsample_rate=1, dropout=0.0, kv_in_dim=None):
        super().__init__()
        self.embedding_dim = embedding_dim
        self.kv_in_dim = kv_in_dim if kv_in_dim is not None else embedding_dim
        self.internal_dim = embedding_dim // downsample_rate
        self.num_heads = num_heads
        assert self.internal_dim % num_heads == 0
        self.q_proj = Linear(embedding_dim, self.internal_dim)
        self.k_proj = Linear(self.kv_in_dim, self.internal_dim)
        self.v_proj = Linear(self.kv_in_dim, self.internal_dim)
        self.out_proj = Linear(self.internal_dim, embedding_dim)
        self.dropout_p = dropout

    def _p(self):
        return self.dropout_p if self.training else 0.0

    def attend(self, q, k, v, residual=None, out_drop=0.0, norm=None):
        """q [B, Lq, I], k/v [B, Lk, I] projected -> out_proj(attn) (+ residual); norm: that sum
        LayerNorm'ed (the post-norm of the two-way blocks, transformer.py:143-187) -- with a residual
        as one full-row GEMM launch with the LayerNorm in its epilogue (FN.linear_add_layer_norm)"""
        B, Lq, I = q.shape
        Lk = k.shape[1]
        h = self.num_heads
        o = FN.attention(q.view(B, Lq, h, I // h), k.view(B, Lk, h, I // h), v.view(B, Lk, h, I // h),
                         p_drop=self._p())
        o3 = o.reshape(B, Lq, I)
        if norm is not None and residual is not None and FN._linear_ln_ok(o3, self.out_proj, norm):
            return FN.linear_add_layer_norm(o3, self.out_proj, residual, norm, norm.eps, drop_p=out_drop)[0]
        y = self.out_proj(o3, residual=residual, drop_p=out_drop)
        return norm(y) if norm is not None else y

    def forward(self, q, k, v, residual=None, norm=None):
        return self.attend(self.q_proj(q), self.k_proj(k), self.v_proj(v), residual=residual, norm=norm)


class RoPEAttention(Attention):
    """transformer.py:251-311"""

    def __init__(self, *args, rope_theta=10000.0, rope_k_repeat=False, feat_sizes=(64, 64), **kwargs):
        super().__init__(*args, **kwargs)
        self.rope_theta = rope_theta
        self.rope_k_repeat = rope_k_repeat
        self.head_dim = self.internal_dim // self.num_heads
        self._vfold = None
        self._vfold_out = None

    def bind_arena(self, arena):
        """the memory cross-attention (kv_in_dim 64, one head of 256) folds its value projection
        into the attention (FN.VFoldProj / ops.attn_fwd_vfold)"""
        if self.kv_in_dim == ops.VFOLD_DV and self.num_heads == 1 and self.internal_dim == 256:
            self._vfold = FN.VFoldProj(self.v_proj)
            self._vfold_out = FN.VFoldOutProj(self._vfold, self.out_proj)

    def attend_mem(self, q, k, mem, residual=None, out_drop=0.0, add_ln=None):
        """attention of projected q / k over the memory bank `mem` [B, Lk, 64] with its value
        projection: out_proj(attn(q, k, v_proj(mem))) (+ residual).  bf16 on the flash path runs the
        V-fold -- softmax(q k^T) (mem Wv^T + bv) = [P mem | rowsum(P)] [Wv | bv]^T: the 64-wide memory
        is streamed instead of its 256-wide projection, which is never formed.  add_ln = (x, norm):
        returns (norm(x + y), x + y) for the output y instead -- the residual add + LayerNorm that
        follows (memory_attention.py:66-94), fused into the output GEMM where it can be."""
        B, Lq, I = q.shape
        Lk = k.shape[1]
        q4 = q.view(B, Lq, 1, I)
        if self._vfold is not None and FN.vfold_enabled() and ops.vfold_ok(q4, mem):
            u = FN.attention_vfold(q4, k.view(B, Lk, 1, I), mem.reshape(B, Lk, 1, mem.shape[-1]), p_drop=self._p())
            if FN.vfold_out_enabled():  # value and output projection as one GEMM (FN.VFoldOutProj)
                u3 = u.view(B, Lq, ops.VFOLD_COLS)
                if add_ln is not None:
                    x, norm = add_ln
                    return FN.linear_add_layer_norm(u3, self._vfold_out, x, norm, norm.eps, drop_p=out_drop)
                return FN.linear(u3, self._vfold_out, residual=residual, drop_p=out_drop)
            o = FN.linear(u.view(B, Lq, ops.VFOLD_COLS), self._vfold)
            if add_ln is not None:
                x, norm = add_ln
                return FN.linear_add_layer_norm(o, self.out_proj, x, norm, norm.eps, drop_p=out_drop)
            return self.out_proj(o, residual=residual, drop_p=out_drop)
        y = self.attend(q, k, self.v_proj(mem), residual=residual, out_drop=out_drop)
        if add_ln is not None:
            x, norm = add_ln
            return FN.add_layer_norm(x, y, norm, norm.eps)
        return y

    def tables(self, Lq, device):
        w = h = math.sqrt(Lq)
        return axial_rope_table(self.head_dim, w, h, self.rope_theta, device)

    def rope_q(self, q, Lq):
        cos, sin = self.tables(Lq, q.device)
        return FN.rope(q, Lq, cos, sin, Lq)

    def proj_q(self, x, Lq):
        """rope_q(q_proj(x)) as one GEMM with the rotation in its epilogue"""
        cos, sin = self.tables(Lq, x.device)
        L = x.shape[1]
        return FN.linear(x, self.q_proj, rope=(cos, sin, L, L, Lq, self.internal_dim, self.head_dim))

    def proj_k(self, x, Lq, num_k_exclude_rope=0):
        """rope_k(k_proj(x), Lq, num_k_exclude_rope) as one GEMM with the rotation in its epilogue
        (the last num_k_exclude_rope rows -- object-pointer tokens -- unrotated)"""
        Lk = x.shape[1]
        nr = Lk - num_k_exclude_rope
        if nr != Lq:
            assert self.rope_k_repeat
        cos, sin = self.tables(Lq, x.device)
        return FN.linear(x, self.k_proj, rope=(cos, sin, Lk, nr, Lq, self.internal_dim, self.head_dim))

    def rope_k(self, k, Lq, num_k_exclude_rope=0):
        nr = k.shape[1] - num_k_exclude_rope
        if nr != Lq:
            assert self.rope_k_repeat
        cos, sin = self.tables(Lq, k.device)
        return FN.rope(k, nr, cos, sin, Lq)

    def forward(self, q, k, v, num_k_exclude_rope=0, residual=None, out_drop=0.0):
        Lq = q.shape[1]
        qp = self.proj_q(q, Lq)
        kp = self.proj_k(k, Lq, num_k_exclude_rope)
        return self.attend(qp, kp, self.v_proj(v), residual=residual, out_drop=out_drop)


class TwoWayAttentionBlock(nn.Module):
    """transformer.py:112-187"""

    def __init__(self, embedding_dim, num_heads, mlp_dim=2048, activation=None, attention_downsample_rate=2,
                 skip_first_layer_pe=False):
        super().__init__()
        self.self_attn = Attention(embedding_dim, num_heads)
        self.norm1 = LayerNorm(embedding_dim)
        self.cross_attn_token_to_image = Attention(embedding_dim, num_heads, downsample_rate=attention_downsample_rate)
        self.norm2 = LayerNorm(embedding_dim)
        self.mlp = MLP(embedding_dim, mlp_dim, embedding_dim, num_layers=2, activation="relu")
        self.norm3 = LayerNorm(embedding_dim)
        self.norm4 = LayerNorm(embedding_dim)
        self.cross_attn_image_to_token = Attention(embedding_dim, num_heads, downsample_rate=attention_downsample_rate)
        self.skip_first_layer_pe = skip_first_layer_pe

    def forward(self, queries, keys, query_pe, key_pe_table):
        # every residual add and the post-norm after it run in the out-projection's epilogue
        # (Attention.attend / MLP norm=: FN.linear_add_layer_norm)
        if self.skip_first_layer_pe:
            queries = self.self_attn(queries, queries, queries, norm=self.norm1)
        else:
            q = FN.add(queries, query_pe)
            queries = self.self_attn(q, q, queries, residual=queries, norm=self.norm1)
        q = FN.add(queries, query_pe)
        k = FN.add_bcast(keys, key_pe_table)
        queries = self.cross_attn_token_to_image(q, k, keys, residual=queries, norm=self.norm2)
        queries = self.mlp(queries, residual=queries, norm=self.norm3)
        q = FN.add(queries, query_pe)
        keys = self.cross_attn_image_to_token(k, q, queries, residual=keys, norm=self.norm4)
        return queries, keys


class TwoWayTransformer(nn.Module):
    """transformer.py:19-109"""

    def __init__(self, depth, embedding_dim, num_heads, mlp_dim, activation=None, attention_downsample_rate=2):
        super().__init__()
        self.depth = depth
        self.layers = nn.ModuleList(
            TwoWayAttentionBlock(embedding_dim, num_heads, mlp_dim, attention_downsample_rate=attention_downsample_rate,
                                 skip_first_layer_pe=(i == 0)) for i in range(depth))
        self.final_attn_token_to_image = Attention(embedding_dim, num_heads, downsample_rate=attention_downsample_rate)
        self.norm_final_attn = LayerNorm(embedding_dim)

    def forward(self, image_embedding, image_pe_table, point_embedding):
        """image_embedding [B, HW, C]; image_pe_table [HW, C] constant; point_embedding [B, T, C]"""
        tape = _ft.active()
        if tape is not None and dec_tok_enabled() and all(_ft.dec_tok_ok(point_embedding, b) for b in self.layers):
            return self._forward_tape_fused(tape, image_embedding, image_pe_table, point_embedding)
        queries, keys = point_embedding, image_embedding
        for layer in self.layers:
            queries, keys = layer(queries, keys, point_embedding, image_pe_table)
        q = FN.add(queries, point_embedding)
        k = FN.add_bcast(keys, image_pe_table)
        queries = self.final_attn_token_to_image(q, k, keys, residual=queries, norm=self.norm_final_attn)
        return queries, keys

    def _forward_tape_fused(self, tape, keys, pe_table, pe):
        """forward() on the frame tape with each block's token side as two launches (csrc/decoder_tok.hip:
        _ft.dec_self before the token -> image attention, _ft.dec_post after it) and the final token side
        as one (_ft.dec_final); the image-side projections, both cross-attentions and norm4 as before.
        The tape records the same ops (the token ones in the order the fused launches compute them)."""
        queries = pe
        n = len(self.layers)
        fa = self.final_attn_token_to_image
        qqf = None
        k_next = None  # keys + key_pe written by the previous block's norm4 launch (_ft.layer_norm_pe)
        for i, blk in enumerate(self.layers):
            t2i, i2t = blk.cross_attn_token_to_image, blk.cross_attn_image_to_token
            x1, qq = _ft.dec_self(tape, queries, pe, blk.self_attn, blk.norm1, t2i.q_proj, blk.skip_first_layer_pe)
            k = k_next if k_next is not None else FN.add_bcast(keys, pe_table)
            B, Lq, I = qq.shape
            Lk, h = k.shape[1], t2i.num_heads
            o = FN.attention(qq.view(B, Lq, h, I // h), t2i.k_proj(k).view(B, Lk, h, I // h),
                             t2i.v_proj(keys).view(B, Lk, h, I // h), p_drop=t2i._p())
            queries, ki, vi, qf = _ft.dec_post(tape, o.reshape(B, Lq, I), x1, pe, t2i.out_proj, blk.norm2, blk.mlp,
                                               blk.norm3, i2t.k_proj, i2t.v_proj, fa.q_proj if i == n - 1 else None)
            if qf is not None:
                qqf = qf
            oi = FN.attention(i2t.q_proj(k).view(B, Lk, h, I // h), ki.view(B, Lq, h, I // h),
                              vi.view(B, Lq, h, I // h), p_drop=i2t._p())
            xk = i2t.out_proj(oi.reshape(B, Lk, I), residual=keys)
            if _ft.layer_norm_pe_ok(xk, blk.norm4, pe_table):  # norm4 and the next k = keys + key_pe: one launch
                keys, k_next = _ft.layer_norm_pe(tape, xk, blk.norm4, blk.norm4.eps, pe_table)
            else:
                keys, k_next = blk.norm4(xk), None
        k = k_next if k_next is not None else FN.add_bcast(keys, pe_table)
        B, Lq, I = qqf.shape
        Lk, h = k.shape[1], fa.num_heads
        o = FN.attention(qqf.view(B, Lq, h, I // h), fa.k_proj(k).view(B, Lk, h, I // h),
                         fa.v_proj(keys).view(B, Lk, h, I // h), p_drop=fa._p())
        queries = _ft.dec_final(tape, o.reshape(B, Lq, I), queries, fa.out_proj, self.norm_final_attn)
        return queries, keys


def dec_tok_enabled():
    """S2H_DEC_TOK=0: the two-way transformer's token side as its separate launches (A/B of
    csrc/decoder_tok.hip)"""
    import os
    return os.environ.get("S2H_DEC_TOK", "1") == "1"
