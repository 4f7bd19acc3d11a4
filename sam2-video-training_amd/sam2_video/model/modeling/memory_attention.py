"""Memory attention (reference memory_attention.py:17-169), batch-first [O, L, C].

Per layer: LN1 -> fused q/k/v GEMM (arena-adjacent weights, RoPE(q, k) in its epilogue) ->
flash attention -> out-proj GEMM with dropout + residual in the epilogue;
LN2 -> q GEMM (+ RoPE in the epilogue), k GEMM on (memory + memory_pos) with RoPE in the
epilogue on the spatial rows (table repeated per memory frame, object-pointer rows excluded), v GEMM on
memory -> flash attention over Lk = n_frames*L + 4*n_ptr -> out-proj (+res) -- in bf16 the value
projection is folded into the attention (RoPEAttention.attend_mem: the 64-wide memory is the
attention's value, [Wv | bv] one GEMM after it);
LN3 -> linear1 (ReLU + dropout in the epilogue) -> linear2 (+dropout, +res).
"""
from __future__ import annotations

import copy
import os

from torch import nn

from ...kernels import functional as FN
from .layers import FusedLinear, LayerNorm, Linear


def shared_qkv_enabled():
    """layer 0's norm1 + q/k/v GEMM once per frame instead of once per object (default on;
    S2H_MA_SHARED_QKV=0 restores the per-object form for A/B)"""
    return os.environ.get("S2H_MA_SHARED_QKV", "1") != "0"


class MemoryAttentionLayer(nn.Module):
    """memory_attention.py:17-99"""

    def __init__(self, activation: str, cross_attention: nn.Module, d_model: int, dim_feedforward: int,
                 dropout: float, pos_enc_at_attn: bool, pos_enc_at_cross_attn_keys: bool,
                 pos_enc_at_cross_attn_queries: bool, self_attention: nn.Module):
        super().__init__()
        assert activation == "relu" and not pos_enc_at_attn and pos_enc_at_cross_attn_keys
        assert not pos_enc_at_cross_attn_queries
        self.d_model = d_model
        self.dim_feedforward = dim_feedforward
        self.dropout_value = dropout
        self.self_attn = self_attention
        self.cross_attn_image = cross_attention
        self.linear1 = Linear(d_model, dim_feedforward)
        self.linear2 = Linear(dim_feedforward, d_model)
        self.norm1 = LayerNorm(d_model)
        self.norm2 = LayerNorm(d_model)
        self.norm3 = LayerNorm(d_model)
        self._fused_qkv = None

    def bind_arena(self, arena):
        sa = self.self_attn
        f = FusedLinear([sa.q_proj, sa.k_proj, sa.v_proj], arena)
        self._fused_qkv = f if f.packed else None

    def arena_groups(self, prefix):
        sa = prefix + ".self_attn"
        return [[f"{sa}.q_proj.weight", f"{sa}.k_proj.weight", f"{sa}.v_proj.weight"],
                [f"{sa}.q_proj.bias", f"{sa}.k_proj.bias", f"{sa}.v_proj.bias"]]

    def _drop(self):
        return self.dropout_value if self.training else 0.0

    def sublayers(self, x, t, mem_k, mem_v, num_k_exclude_rope, next_norm):
        """The layer on the residual stream x with t = norm1(x) given; returns (x', next_norm(x')).
        t may hold ONE object's rows ([1, L, C]) when every object's stream is the same (layer 0: the
        current frame's features broadcast to the objects) -- then the q/k/v projection runs once and
        its output is broadcast (its gradient summed over the objects) instead of running per object.
        Every residual add is fused with the LayerNorm that reads its result, and (bf16) with the
        projection that produces it: FN.linear_add_layer_norm runs out_proj / the folded
        cross-attention output / linear2, dropout, the residual add and the next LayerNorm as ONE
        full-row GEMM launch (LN(x + y) and x + y; in the backward LN'(.) + the stream's gradient in
        one pass), so each residual state has a single autograd consumer and no separate
        gradient-accumulation adds run (memory_attention.py:58-99 order and dropouts)."""
        L = x.shape[1]
        C = self.d_model
        p = self._drop()
        sa = self.self_attn
        if self._fused_qkv is not None and sa.num_heads == 1:
            # one q/k/v GEMM with q and k rotated in its epilogue; out_proj + residual + norm2 as one
            # full-row GEMM with the LayerNorm in its epilogue (FN.linear_add_layer_norm)
            cos, sin = sa.tables(L, t.device)
            qkv = self._fused_qkv(t, rope=(cos, sin, L, L, L, 2 * C, C))
            if qkv.shape[0] != x.shape[0]:
                qkv = FN.expand_batch(qkv, x.shape[0])
            o = FN.qkv_attention(qkv.view(qkv.shape[0], L, 3, 1, C), p_drop=sa._p())
            t, x = FN.linear_add_layer_norm(o.reshape(qkv.shape[0], L, C), sa.out_proj, x, self.norm2,
                                            self.norm2.eps, drop_p=p)
        else:
            if t.shape[0] != x.shape[0]:
                t = FN.expand_batch(t, x.shape[0])
            q = sa.proj_q(t, L)
            k = sa.proj_k(t, L)
            y = sa.attend(q, k, sa.v_proj(t), out_drop=p)
            t, x = FN.add_layer_norm(x, y, self.norm2, self.norm2.eps)
        ca = self.cross_attn_image
        q = ca.proj_q(t, L)
        k = ca.proj_k(mem_k, L, num_k_exclude_rope)
        t, x = ca.attend_mem(q, k, mem_v, out_drop=p, add_ln=(x, self.norm3))
        if FN._linear_ln_ok(t, self.linear2, next_norm):  # opt-in full-row linear2 + add + LayerNorm
            h = self.linear1(t, act="relu", drop_p=p)
            t, x = FN.linear_add_layer_norm(h, self.linear2, x, next_norm, next_norm.eps, drop_p=p)
        else:  # both FFN GEMMs as one launch on the frame tape (FN.ffn), then add + LayerNorm
            t, x = FN.add_layer_norm(x, FN.ffn(t, self.linear1, self.linear2, p), next_norm, next_norm.eps)
        return x, t

    def forward(self, tgt, mem_k, mem_v, num_k_exclude_rope=0):
        L = tgt.shape[1]
        C = self.d_model
        p = self._drop()
        # self-attention (:58-64), q = k = v = norm1(tgt), RoPE on q and k
        sa = self.self_attn
        t2 = self.norm1(tgt)
        if self._fused_qkv is not None and sa.num_heads == 1:
            # one packed q/k/v GEMM with q and k rotated in its epilogue; the attention reads it in
            # place and the backward returns one packed gradient (FN.qkv_attention)
            cos, sin = sa.tables(L, t2.device)
            qkv = self._fused_qkv(t2, rope=(cos, sin, L, L, L, 2 * C, C))
            o = FN.qkv_attention(qkv.view(qkv.shape[0], L, 3, 1, C), p_drop=sa._p())
            tgt = sa.out_proj(o.reshape(qkv.shape[0], L, C), residual=tgt, drop_p=p)
        else:
            q, k, v = sa.proj_q(t2, L), sa.proj_k(t2, L), sa.v_proj(t2)
            tgt = sa.attend(q, k, v, residual=tgt, out_drop=p)
        # cross-attention to the memory bank (:66-81)
        ca = self.cross_attn_image
        t2 = self.norm2(tgt)
        q = ca.proj_q(t2, L)
        k = ca.proj_k(mem_k, L, num_k_exclude_rope)
        tgt = ca.attend_mem(q, k, mem_v, residual=tgt, out_drop=p)
        # feed-forward (:95-98)
        t2 = self.norm3(tgt)
        h = self.linear1(t2, act="relu", drop_p=p)
        return self.linear2(h, residual=tgt, drop_p=p)


class MemoryAttention(nn.Module):
    """memory_attention.py:102-169"""

    def __init__(self, d_model: int, pos_enc_at_input: bool, layer: nn.Module, num_layers: int,
                 batch_first: bool = True):
        super().__init__()
        self.d_model = d_model
        self.layers = nn.ModuleList([copy.deepcopy(layer) for _ in range(num_layers)])
        self.num_layers = num_layers
        self.norm = LayerNorm(d_model)
        self.pos_enc_at_input = pos_enc_at_input
        self.batch_first = batch_first

    def forward(self, curr, curr_pos, memory, memory_pos_table, num_obj_ptr_tokens=0, num_objects=1):
        """curr [L, C] (one frame, shared by all objects), curr_pos [L, C] constant,
        memory [O, M, 64] (detached bank), memory_pos_table [M, 64] (shared by objects)
        -> [O, L, C]"""
        x = FN.add(curr, curr_pos, beta=0.1) if self.pos_enc_at_input else curr
        x1 = x.unsqueeze(0)
        x = FN.expand_batch(x1, num_objects)
        mem_k = FN.add_bcast(memory, memory_pos_table)
        # layer 0's LN1 (and q/k/v projection, MemoryAttentionLayer.sublayers) on the one shared frame
        t = self.layers[0].norm1(x1 if shared_qkv_enabled() else x)
        for i, layer in enumerate(self.layers):
            nxt = self.layers[i + 1].norm1 if i + 1 < len(self.layers) else self.norm
            x, t = layer.sublayers(x, t, mem_k, memory, num_obj_ptr_tokens, nxt)
        return t  # = self.norm(x) (memory_attention.py:167)
