"""Autograd functions over libsam2hip kernels.

Weights live in the flat fp32 parameter arena (sam2_video.kernels.arena): every
weight-carrying module exposes `.w` (compute-dtype weight), `.b` (fp32 bias) and
writes its gradients straight into `param._s2h_grad` (a view of the flat fp32
gradient arena) inside backward, returning None to autograd.  The Parameter is
still passed as an input so autograd builds the node whenever the parameter is
trainable, even when the activation does not require grad.

Every op here launches HIP kernels only (no torch arithmetic on the data path);
torch provides allocation, views and the autograd tape.
"""
from __future__ import annotations

import math
import os

import torch

from . import fp8 as _fp8
from . import frametape as _ft
from . import ops

_SEED = [0x5EED]


def next_seed():
    _SEED[0] = (_SEED[0] * 6364136223846793005 + 1442695040888963407) & (2**64 - 1)
    return _SEED[0]


def set_seed(s):
    _SEED[0] = int(s) & (2**64 - 1)


# weight generation: bumped once per step (SAM2Model.forward_image); weights derived from the
# arena (the folded value projection) are rebuilt on their first use in a new generation -- inside
# the step, so a captured graph rebuilds them on every replay
_GEN = [0]


def new_step():
    _GEN[0] += 1


def _compute_weight(mod):
    """a Linear / Conv2d module's weight in the compute dtype as a [out, in*k*k] matrix"""
    return mod.weight._s2h_compute.reshape(mod.weight.shape[0], -1)


def _grad_of(p):
    return getattr(p, "_s2h_grad", None) if p is not None and p.requires_grad else None


# ---------------------------------------------------------------- Linear
class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, wp, bp, mod, act, residual, drop_p, rope=None):
        w = mod.compute_weight()
        b = mod.compute_bias()
        ctx.rope = rope
        if rope is not None:  # RoPE of the output in the GEMM epilogue (no act / residual / dropout)
            assert act is None and residual is None and drop_p == 0
            out = _fp8.linear_rope(x, mod, w, b, rope)
            ctx.mod, ctx.act, ctx.drop_p, ctx.seed, ctx.relu_out, ctx.has_res = mod, None, 0.0, 0, False, False
            ctx.save_for_backward(x, None)
            return out
        # ReLU without residual: the backward masks with the output itself (no pre-activation)
        relu_out = act == "relu" and residual is None
        pre = torch.empty(*x.shape[:-1], w.shape[0], device=x.device, dtype=x.dtype) if act and not relu_out else None
        seed = next_seed() if drop_p > 0 else 0
        out = _fp8.linear(x, mod, w, b, act=act, pre=pre, residual=residual, drop_p=drop_p, seed=seed)
        ctx.mod, ctx.act, ctx.drop_p, ctx.seed, ctx.relu_out = mod, act, drop_p, seed, relu_out
        ctx.has_res = residual is not None
        ctx.save_for_backward(x, out if relu_out else pre)
        return out

    @staticmethod
    def backward(ctx, dy):
        x, pre = ctx.saved_tensors
        mod = ctx.mod
        dy = dy.contiguous()
        if ctx.rope is not None:  # the gradient of the rotated output, rotated back (in place)
            ops.rope_blocks(dy.view(-1, dy.shape[-1]), ctx.rope, inverse=True)
        if ctx.relu_out:
            dpre = ops.relu_mask_bwd(pre, dy, 1.0 / (1.0 - ctx.drop_p))
        elif ctx.drop_p > 0:
            dpre = ops.act_dropout_bwd(pre if ctx.act else None, dy, ctx.act, ctx.drop_p, ctx.seed)
        else:
            dpre = ops.act_bwd(pre, dy, ctx.act) if ctx.act else dy
        wgrad = getattr(mod, "wgrad", None)
        gw, gb = mod.grad_views()
        if wgrad is not None:
            wgrad(dpre, x)
        elif gw is not None:
            ops.linear_wgrad(dpre, x, gw.view(gw.shape[0], -1), db=gb)
        elif gb is not None:
            ops.colsum(dpre, gb)
        dx = _fp8.linear_dgrad(dpre, mod) if ctx.needs_input_grad[0] else None
        return dx, None, None, None, None, (dy if ctx.has_res else None), None, None


def linear(x, mod, act=None, residual=None, drop_p=0.0, rope=None):
    """drop(act(x @ W^T + b)) (+ residual).  `mod` provides compute_weight(), compute_bias(),
    grad_views() and `weight`/`bias` anchors (Parameters) for the autograd tape.  rope = (cos, sin,
    L, nrot, period, ncol, dh): the output rotated by the axial RoPE in the GEMM epilogue
    (ops.rope_blocks layout; no act / residual / dropout)."""
    T = _ft.active()
    if T is not None:
        return _ft.linear(T, x, mod, act, residual, float(drop_p), rope=rope)
    # a 2-D input with contiguous rows keeps its row pitch (the patch embedding's im2col matrix: 147
    # columns in 152-element rows, so its weight gradient stays on the LDS-DMA kernel)
    if not (x.dim() == 2 and x.stride(1) == 1 and x.stride(0) >= x.shape[1]):
        x = x.contiguous()
    return _Linear.apply(x, mod.weight, mod.bias, mod, act, residual, float(drop_p), rope)


class _MLP2(torch.autograd.Function):
    """fc2(act(fc1(x))) (+ residual) as one node: the backward applies act'(pre) in fc2's dgrad
    epilogue (no separate activation-gradient pass, no d(hidden) round trip through HBM)."""

    @staticmethod
    def forward(ctx, x, w1p, b1p, w2p, b2p, fc1, fc2, act, residual):
        w1, w2 = fc1.compute_weight(), fc2.compute_weight()
        pre = torch.empty(*x.shape[:-1], w1.shape[0], device=x.device, dtype=x.dtype)
        hid = _fp8.linear(x, fc1, w1, fc1.compute_bias(), act=act, pre=pre)
        out = _fp8.linear(hid, fc2, w2, fc2.compute_bias(), residual=residual)
        ctx.fc1, ctx.fc2, ctx.act, ctx.has_res = fc1, fc2, act, residual is not None
        ctx.save_for_backward(x, pre, hid)
        return out

    @staticmethod
    def backward(ctx, dy):
        x, pre, hid = ctx.saved_tensors
        dy = dy.contiguous()
        fc1, fc2 = ctx.fc1, ctx.fc2
        gw2, gb2 = fc2.grad_views()
        if gw2 is not None:
            ops.linear_wgrad(dy, hid, gw2.view(gw2.shape[0], -1), db=gb2)
        elif gb2 is not None:
            ops.colsum(dy, gb2)
        dpre = _fp8.linear_dgrad(dy, fc2, pre=pre, act=ctx.act)
        gw1, gb1 = fc1.grad_views()
        if gw1 is not None:
            ops.linear_wgrad(dpre, x, gw1.view(gw1.shape[0], -1), db=gb1)
        elif gb1 is not None:
            ops.colsum(dpre, gb1)
        dx = _fp8.linear_dgrad(dpre, fc1) if ctx.needs_input_grad[0] else None
        return dx, None, None, None, None, None, None, None, (dy if ctx.has_res else None)


def mlp2(x, fc1, fc2, act, residual=None):
    """fc2(act(fc1(x))) (+ residual) -- two-layer MLP (hieradet.py:87-91 MultiScaleBlock.mlp)"""
    T = _ft.active()
    if T is not None:
        return linear(linear(x, fc1, act=act), fc2, residual=residual)
    return _MLP2.apply(x.contiguous(), fc1.weight, fc1.bias, fc2.weight, fc2.bias, fc1, fc2, act, residual)


# ------------------------------------------------------------- LayerNorm
class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gp, bp, mod, eps, add, add_bcast):
        xsum = torch.empty_like(x) if add is not None else None
        y, mean, rstd = ops.layernorm_fwd(x, gp.detach(), bp.detach(), eps, add=add, add_bcast=add_bcast, xsum=xsum)
        ctx.mod = mod
        ctx.has_add = add is not None
        ctx.add_bcast = add_bcast
        ctx.save_for_backward(xsum if add is not None else x, mean, rstd)
        if add is not None:
            return y, xsum
        return y

    @staticmethod
    def backward(ctx, dy, dxsum=None):
        x, mean, rstd = ctx.saved_tensors
        mod = ctx.mod
        dy = dy.contiguous()
        gw, gb = _grad_of(mod.weight), _grad_of(mod.bias)
        dx = None
        if dxsum is not None:
            dx = ops.layernorm_bwd(x, dy, mod.weight.detach(), mean, rstd, dres=dxsum.contiguous(), dgamma=gw, dbeta=gb)
        else:
            dx = ops.layernorm_bwd(x, dy, mod.weight.detach(), mean, rstd, dgamma=gw, dbeta=gb)
        dadd = None
        if ctx.has_add:
            if ctx.add_bcast:
                dadd = None  # broadcast adds are constants (positional encodings)
            else:
                dadd = dx
        return dx, None, None, None, None, dadd, None


def layer_norm(x, mod, eps):
    T = _ft.active()
    if T is not None:
        return _ft.layer_norm(T, x, mod, eps)
    return _LayerNorm.apply(x.contiguous(), mod.weight, mod.bias, mod, eps, None, False)


def add_layer_norm(x, add, mod, eps):
    """returns (LN(x + add), x + add) -- fused residual add + norm"""
    T = _ft.active()
    if T is not None:
        return _ft.layer_norm(T, x, mod, eps, add=add if add.is_contiguous() else add.contiguous())
    return _LayerNorm.apply(x.contiguous(), mod.weight, mod.bias, mod, eps, add.contiguous(), False)


# ------------------------------------------------ no-grad per-object MLP heads (one launch)
def _head_ok(m, x):
    layers = getattr(m, "layers", None)
    if layers is None or getattr(m, "act", None) != "relu" or not (1 <= len(layers) <= 3):
        return False
    if x.dtype != torch.bfloat16 or x.dim() != 2 or x.stride(1) != 1 or x.stride(0) % 8 or x.data_ptr() % 16:
        return False
    k = x.shape[1]
    for i, lin in enumerate(layers):
        w = lin.compute_weight()
        last = i == len(layers) - 1
        if w.dtype != torch.bfloat16 or not w.is_contiguous() or w.shape[1] != k or k > 256 or k % 8 or \
                w.shape[0] > 256 or (not last and w.shape[0] % 8) or w.data_ptr() % 16:
            return False
        k = w.shape[0]
    return True


def _heads_fusable(pairs):
    import os
    return (0 < len(pairs) <= 4 and os.environ.get("S2H_MLP_HEADS", "1") != "0"
            and len({x.shape[0] for _, x in pairs}) == 1 and all(_head_ok(m, x) for m, x in pairs))


def mlp_heads(pairs):
    """[(MLP module, x [M, K] rows)] -> [module(x)] for the decoder's trained per-object heads (the
    hypernetwork MLP of mask token 0 and the IoU head, mask_decoder.py:227-233): in the frame tape one
    launch for all of them with the hidden activations saved for the frame-batched backward
    (frametape.mlp_heads); without autograd the no-grad launch; else each head's own forward"""
    if not torch.is_grad_enabled():
        return mlp_heads_nograd(pairs)
    T = _ft.active()
    if T is not None and _heads_fusable(pairs):
        return _ft.mlp_heads(T, pairs)
    return [m(x) for m, x in pairs]


def mlp_heads_nograd(pairs):
    """[(MLP module, x [M, K] rows)] -> [module(x)] for heads whose outputs need no gradient (the object
    score head, mask_decoder.py:234-238, and the object-pointer projection, sam2_base.py:296-305): one
    launch for all of them (s2h_mlp_heads: per head the layers chained in LDS, bit-identical to the
    per-layer GEMMs) when every head is a bf16 ReLU MLP of <= 3 layers no wider than 256; else each
    head's own forward.  S2H_MLP_HEADS=0 keeps the per-layer GEMMs (A/B)."""
    if not _heads_fusable(pairs):
        return [m(x) for m, x in pairs]
    return ops.mlp_heads([(x, [lin.compute_weight() for lin in m.layers], [lin.compute_bias() for lin in m.layers],
                           "sigmoid" if m.sigmoid_output else None) for m, x in pairs])


# ------------------------------------------------ Linear + residual add + LayerNorm (one launch)
def ffn_fwd_enabled():
    """S2H_FFN_FWD=1 runs the memory-attention FFN forward as one ops.ffn_fwd launch instead of its two
    Linear launches.  Off by default: at a tracked frame's 13 312 rows the fused kernel has 208 one-per-CU
    workgroups and its ReLU / dropout-hash epilogue runs with the MFMA pipes idle -- 73.7 us per launch
    against 70.5 us for the two GEMMs (graph-replayed, tools/ffn_bench.py, profiles/r05_ffn_bench.log),
    bench step 153.0 / 152.8 vs 154.4 / 154.3 clip-frames/s (profiles/r05_v8_ffn_fwd_ab.log)"""
    import os
    return os.environ.get("S2H_FFN_FWD", "0") == "1"


def ffn(x, mod1, mod2, drop_p=0.0):
    """drop(linear2(drop(relu(linear1(x))))) (memory_attention.py:97): on the frame tape one launch
    (_ft.ffn: the two Linear ops recorded as such, ops.ffn_fwd computing both), else the two Linears"""
    T = _ft.active()
    if T is not None and ffn_fwd_enabled() and _ft.ffn_fwd_ok(x, mod1, mod2):
        return _ft.ffn(T, x if x.is_contiguous() else x.contiguous(), mod1, mod2, float(drop_p))
    return linear(linear(x, mod1, act="relu", drop_p=drop_p), mod2, drop_p=drop_p)


def linear_ln_enabled():
    """S2H_LINEAR_LN=1 runs a projection + the residual add + LayerNorm after it as ONE full-row GEMM
    launch.  Off by default: on MI355X the 64 x 256 full-row tile (160 KB of LDS, one workgroup per
    CU, the whole weight re-read per 64 rows) is slower than the 64 x 64 tile plus a LayerNorm launch
    (profiles/r04_v3_fullrow_tiles.log; bench step 57.8 ms unfused vs 59.6 ms fused,
    profiles/r04_v3_ln_fusion_ab.log)"""
    import os
    return os.environ.get("S2H_LINEAR_LN", "0") == "1"


def _linear_ln_ok(inp, mod, norm):
    N = mod.out_features
    return (linear_ln_enabled() and inp.dtype == torch.bfloat16 and N in (128, 256) and norm.weight.shape[0] == N
            and inp.shape[-1] % 8 == 0 and not (_fp8._eligible(mod) and _fp8._pays(inp.shape[-1], N)))


class _LinearAddLN(torch.autograd.Function):
    """(LN(x + drop(inp W^T + b)), x + drop(inp W^T + b)) from one full-row GEMM launch
    (ops.linear_add_ln); backward: the LayerNorm backward (with the residual stream's gradient) and
    the linear backward of its result"""

    @staticmethod
    def forward(ctx, inp, wp, bp, x, gp, gbp, mod, norm, eps, drop_p):
        seed = next_seed() if drop_p > 0 else 0
        t, xsum, mean, rstd = ops.linear_add_ln(inp, mod.compute_weight(), mod.compute_bias(), x, gp.detach(),
                                                gbp.detach(), eps, drop_p=drop_p, seed=seed)
        ctx.mod, ctx.norm, ctx.drop_p, ctx.seed = mod, norm, drop_p, seed
        ctx.save_for_backward(inp, xsum, mean, rstd)
        return t, xsum

    @staticmethod
    def backward(ctx, dt, dxsum):
        inp, xsum, mean, rstd = ctx.saved_tensors
        mod, norm = ctx.mod, ctx.norm
        dt = torch.zeros_like(xsum) if dt is None else dt.contiguous()
        dsum = ops.layernorm_bwd(xsum, dt, norm.weight.detach(), mean, rstd,
                                 dres=dxsum.contiguous() if dxsum is not None else None,
                                 dgamma=_grad_of(norm.weight), dbeta=_grad_of(norm.bias))
        dpre = ops.act_dropout_bwd(None, dsum, None, ctx.drop_p, ctx.seed) if ctx.drop_p > 0 else dsum
        wgrad = getattr(mod, "wgrad", None)
        gw, gb = mod.grad_views()
        if wgrad is not None:
            wgrad(dpre, inp)
        elif gw is not None:
            ops.linear_wgrad(dpre, inp, gw.view(gw.shape[0], -1), db=gb)
        elif gb is not None:
            ops.colsum(dpre, gb)
        dinp = _fp8.linear_dgrad(dpre, mod) if ctx.needs_input_grad[0] else None
        return dinp, None, None, (dsum if ctx.needs_input_grad[3] else None), None, None, None, None, None, None


def linear_add_layer_norm(inp, mod, x, norm, eps, drop_p=0.0):
    """(LN(x + y), x + y) with y = drop(inp W^T + b): a projection followed by the residual add +
    LayerNorm that reads it (memory_attention.py:60-98).  bf16 with a 128 / 256-wide output: one
    full-row GEMM launch with the LayerNorm in its epilogue (s2h_linear_add_ln); else linear +
    add_layer_norm."""
    if not _linear_ln_ok(inp, mod, norm):
        return add_layer_norm(x, linear(inp, mod, drop_p=drop_p), norm, eps)
    T = _ft.active()
    if T is not None:
        return _ft.linear_add_ln(T, inp, mod, x, norm, eps, float(drop_p))
    return _LinearAddLN.apply(inp.contiguous(), mod.weight, mod.bias, x.contiguous(), norm.weight, norm.bias, mod, norm,
                              eps, float(drop_p))


# ------------------------------------------------------------- attention
def _keep_buffer(ctx, q, Lk, p_drop, nin):
    """dropout keep bitmap of a training attention on the flash path (the backward reads it
    instead of re-hashing every element); None otherwise"""
    if not any(ctx.needs_input_grad[:nin]) or not ops.keep_bits_ok(q, p_drop):
        return None
    B, Lq, H, _ = q.shape
    return torch.empty(ops.keep_words(B, H, Lq, Lk), device=q.device, dtype=torch.int32)


class _Attention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, scale, p_drop):
        B, Lq, H, D = q.shape
        o = torch.empty(B, Lq, H, D, device=q.device, dtype=q.dtype)
        lse = torch.empty(B, H, Lq, device=q.device, dtype=torch.float32)
        seed = next_seed() if p_drop > 0 else 0
        keep = _keep_buffer(ctx, q, k.shape[1], p_drop, 3)
        ops.attn_fwd(q, k, v, o, lse, scale, p_drop, seed, keep=keep)
        ctx.scale, ctx.p, ctx.seed, ctx.keep = scale, p_drop, seed, keep
        ctx.save_for_backward(q, k, v, o, lse)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        do = do.contiguous()
        dq = torch.empty(q.shape, device=q.device, dtype=q.dtype)
        dk = torch.empty(k.shape, device=k.device, dtype=k.dtype)
        dv = torch.empty(v.shape, device=v.device, dtype=v.dtype)
        ops.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, ctx.scale, ctx.p, ctx.seed, keep=ctx.keep)
        ctx.keep = None
        return dq, dk, dv, None, None


class VFoldProj:
    """The value projection of a folded cross-attention (ops.attn_fwd_vfold) as the weight of ONE
    GEMM: O = u' [Wv | bv | 0]^T over u' = [D M | rowsum(D) | 0] (72 columns), which equals
    D (M Wv^T + bv) -- the reference's v_proj followed by the attention's P V
    (transformer.py:296-307).  The [N, 72] bf16 weight is rebuilt from the arena on first use in
    each step (new_step); its fp32 gradient dO^T u' is scattered back into the Linear's own weight
    and bias gradients (`wgrad`, called by the linear backward in place of grad_views)."""

    def __init__(self, lin):
        self.lin = lin
        self.weight, self.bias = lin.weight, lin.bias  # autograd anchors (the Linear's parameters)
        self.out_features, self.in_features = lin.out_features, ops.VFOLD_COLS
        self._w = None
        self._g = None
        self._gen = -1

    def compute_weight(self):
        if self._gen != _GEN[0]:
            self._w = ops.vfold_weight(self.lin.compute_weight(), self.lin.bias.detach(), out=self._w)
            self._gen = _GEN[0]
        return self._w

    def compute_bias(self):
        return None

    def grad_views(self):
        return None, None

    def wgrad(self, dy, x):
        gw, gb = _grad_of(self.lin.weight), _grad_of(self.lin.bias)
        if gw is None and gb is None:
            return
        if self._g is None:
            self._g = torch.empty(self.out_features, self.in_features, device=dy.device, dtype=torch.float32)
        ops.linear_wgrad(dy, x, self._g, accumulate=False)
        ops.vfold_grad(self._g, gw, gb)


class VFoldOutProj:
    """The folded cross-attention's value projection AND its output projection as ONE GEMM:
    Y = O Wo^T + bo with O = u' V^T (V = [Wv | bv | 0], VFoldProj) is u' (Wo V)^T + bo, so the
    [N, 72] weight W' = Wo V (a 256 x 72 x 256 GEMM per step) replaces the [rows, 256] x [256, 256]
    out-projection GEMM of every layer and frame, and O is never formed (transformer.py:296-311 +
    memory_attention.py:66-81).  Backward: du' = dY W' is the linear's dgrad; the weight gradients
    follow from G = dY^T u' ([N, 72], fp32): dWo += G V^T, dV = Wo^T G (scattered into dWv / dbv by
    ops.vfold_grad), dbo += colsum(dY).  Used by RoPEAttention.attend_mem (S2H_VFOLD_OUT=0: the two
    GEMMs, for A/B)."""

    def __init__(self, vfold, out_lin):
        self.vf, self.out = vfold, out_lin
        self.weight, self.bias = out_lin.weight, out_lin.bias  # autograd anchors (v_proj's ride along)
        self.out_features, self.in_features = out_lin.out_features, ops.VFOLD_COLS
        self._w = None
        self._g = self._v32 = self._wo32 = self._dv = None
        self._gen = -1

    def compute_weight(self):
        if self._gen != _GEN[0]:
            v = self.vf.compute_weight()   # [Nv, 72] bf16 (Nv = Wo's in_features)
            wo = self.out.compute_weight()  # [N, Nv] bf16
            N, Nv = wo.shape
            if self._w is None:
                self._w = torch.empty(N, ops.VFOLD_COLS, device=wo.device, dtype=wo.dtype)
            ops.gemm(wo, v, self._w, M=N, N=ops.VFOLD_COLS, K=Nv, lda_m=Nv, lda_k=1, ldb_k=ops.VFOLD_COLS, ldb_n=1,
                     ldc=ops.VFOLD_COLS)
            self._gen = _GEN[0]
        return self._w

    def compute_bias(self):
        return self.out.compute_bias()

    def grad_views(self):
        return None, None

    def wgrad(self, dy, x):
        gwo, gbo = _grad_of(self.out.weight), _grad_of(self.out.bias)
        gwv, gbv = _grad_of(self.vf.lin.weight), _grad_of(self.vf.lin.bias)
        if gbo is not None:
            ops.colsum(dy, gbo)
        if gwo is None and gwv is None and gbv is None:
            return
        N, C = self.out_features, ops.VFOLD_COLS
        v = self.vf.compute_weight()  # [Nv, 72]
        wo = self.out.compute_weight()  # [N, Nv]
        Nv = wo.shape[1]
        if self._g is None:
            f32 = dict(device=dy.device, dtype=torch.float32)
            self._g = torch.empty(N, C, **f32)
            # G stays fp32 for the two small products below (no bf16 rounding of the weight
            # gradients' common factor; the reference takes dWo, dWv from fp32 accumulations):
            # fp32 copies of the bf16 operands V and Wo, exact fp32 MFMA products
            self._v32 = torch.empty(Nv, C, **f32)
            self._wo32 = torch.empty(N, Nv, **f32)
        ops.linear_wgrad(dy, x, self._g, accumulate=False)  # G = dY^T u'
        ops.cast(v, torch.float32, out=self._v32)
        ops.cast(wo, torch.float32, out=self._wo32)
        if gwo is not None:  # dWo += G V^T
            ops.gemm(self._g, self._v32, gwo.view(N, Nv), M=N, N=Nv, K=C, lda_m=C, lda_k=1, ldb_k=1, ldb_n=C,
                     ldc=Nv, beta=1.0)
        if gwv is not None or gbv is not None:  # dV = Wo^T G -> dWv, dbv
            if self._dv is None:
                self._dv = torch.empty(Nv, C, device=dy.device, dtype=torch.float32)
            ops.gemm(self._wo32, self._g, self._dv, M=Nv, N=C, K=N, lda_m=1, lda_k=Nv, ldb_k=C, ldb_n=1, ldc=C)
            ops.vfold_grad(self._dv, gwv, gbv)


def vfold_out_enabled():
    """S2H_VFOLD_OUT=0 keeps the V-fold projection and the output projection as two GEMMs (A/B)"""
    import os
    return os.environ.get("S2H_VFOLD_OUT", "1") != "0"


def vfold_enabled():
    """S2H_VFOLD=0 keeps the unfolded value projection + attention (A/B measurements)"""
    import os
    return os.environ.get("S2H_VFOLD", "1") != "0"


class _AttentionVFold(torch.autograd.Function):
    """u' = [D M | rowsum(D) | 0] of the folded cross-attention (ops.attn_fwd_vfold); backward:
    the frame-batched V-fold flash backward with one frame.  The memory M is detached (no dM)."""

    @staticmethod
    def forward(ctx, q, k, mem, scale, p_drop):
        B, Lq = q.shape[0], q.shape[1]
        Lk = k.shape[1]
        u = torch.empty(B, Lq, 1, ops.VFOLD_COLS, device=q.device, dtype=q.dtype)
        lse = torch.empty(B, 1, Lq, device=q.device, dtype=torch.float32)
        seed = next_seed() if p_drop > 0 else 0
        keep = _keep_buffer(ctx, q, Lk, p_drop, 2)
        ops.attn_fwd_vfold(q, k, mem, u, lse, scale, p_drop, seed, keep=keep)
        ctx.scale, ctx.p, ctx.seed, ctx.keep = scale, p_drop, seed, keep
        ctx.save_for_backward(q, k, mem, u, lse)
        return u

    @staticmethod
    def backward(ctx, du):
        q, k, mem, u, lse = ctx.saved_tensors
        B, Lq, _, D = q.shape
        Lk = k.shape[1]
        dq = torch.empty(q.shape, device=q.device, dtype=q.dtype)
        dk = torch.empty(B * Lk, 1, D, device=k.device, dtype=k.dtype)
        ops.flash_bwd_frames_vfold(1, B, [Lk], [0], [0], q, k.reshape(B * Lk, 1, D), mem.reshape(B * Lk, 1, -1), u,
                                   du.contiguous(), lse, dq, dk, ctx.scale, ctx.p, ctx.seed, keep=ctx.keep,
                                   koff=[0] if ctx.keep is not None else None)
        ctx.keep = None
        return dq, dk.view(k.shape), None, None, None


def attention_vfold(q, k, mem, scale=None, p_drop=0.0):
    """u' = [D mem | rowsum(D) | 0] with D = dropout(softmax(scale q k^T)): q [B, Lq, 1, 256], k
    [B, Lk, 1, 256], mem [B, Lk, 1, 64] -> [B, Lq, 1, 72] (the folded cross-attention; VFoldProj
    finishes it)"""
    if scale is None:
        scale = 1.0 / math.sqrt(q.shape[-1])
    T = _ft.active()
    if T is not None:
        return _ft.attention_vfold(T, q, k, mem, float(scale), float(p_drop))
    return _AttentionVFold.apply(q, k.contiguous(), mem.contiguous(), float(scale), float(p_drop))


def attention(q, k, v, scale=None, p_drop=0.0):
    """softmax(scale q k^T) v over [B, L, H, D] views (head dim contiguous)."""
    if scale is None:
        scale = 1.0 / math.sqrt(q.shape[-1])
    T = _ft.active()
    if T is not None:
        return _ft.attention(T, q, k, v, float(scale), float(p_drop))
    return _Attention.apply(q, k, v, float(scale), float(p_drop))


class _QKVAttention(torch.autograd.Function):
    """Self-attention straight from a packed projection output qkv [B, L, 3, H, d] (q, k, v of a
    token adjacent, as the fused q/k/v GEMM writes them), optional RoPE on q and k (rope =
    (cos, sin, period), single head: memory-attention self-attention, transformer.py:275-311).
    The backward writes dq, dk, dv into ONE [B, L, 3, H, d] gradient through strided kernel
    outputs (inverse RoPE in place): with three separate slice inputs autograd zero-fills a
    qkv-sized buffer per slice and adds them (3 fills + 3 copies + 2 adds per attention)."""

    @staticmethod
    def forward(ctx, qkv, scale, p_drop, rope):
        B, L, _, H, D = qkv.shape
        q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        if rope is not None:
            cos, sin, period = rope
            qk = torch.empty(B, L, 2, H, D, device=qkv.device, dtype=qkv.dtype)
            ops.rope(q.reshape(B, L, H * D) if q.is_contiguous() else q.view(B, L, H * D), qk[:, :, 0].view(B, L, H * D),
                     L, cos, sin, period)
            ops.rope(k.view(B, L, H * D), qk[:, :, 1].view(B, L, H * D), L, cos, sin, period)
            q, k = qk[:, :, 0], qk[:, :, 1]
        o = torch.empty(B, L, H, D, device=qkv.device, dtype=qkv.dtype)
        lse = torch.empty(B, H, L, device=qkv.device, dtype=torch.float32)
        seed = next_seed() if p_drop > 0 else 0
        keep = _keep_buffer(ctx, q, L, p_drop, 1)
        ops.attn_fwd(q, k, v, o, lse, scale, p_drop, seed, keep=keep)
        ctx.scale, ctx.p, ctx.seed, ctx.rope, ctx.keep = scale, p_drop, seed, rope, keep
        ctx.save_for_backward(qkv, qk if rope is not None else qkv, o, lse)
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, qk, o, lse = ctx.saved_tensors
        B, L, _, H, D = qkv.shape
        q, k = qk[:, :, 0], qk[:, :, 1]
        v = qkv[:, :, 2]
        dqkv = torch.empty(qkv.shape, device=qkv.device, dtype=qkv.dtype)
        dq, dk, dv = dqkv[:, :, 0], dqkv[:, :, 1], dqkv[:, :, 2]
        ops.attn_bwd(q, k, v, o, do.contiguous(), lse, dq, dk, dv, ctx.scale, ctx.p, ctx.seed, keep=ctx.keep)
        ctx.keep = None
        if ctx.rope is not None:
            cos, sin, period = ctx.rope
            for g in (dq, dk):
                g3 = g.view(B, L, H * D)
                ops.rope(g3, g3, L, cos, sin, period, inverse=True)
        return dqkv, None, None, None


class _PoolQKVAttention(torch.autograd.Function):
    """Hiera query-pooling attention (hieradet.py:56-81 with q_pool): q = 2x2 max-pool of the q
    third of the fused qkv [B, H, W, 3d] projection, k / v read in place.  The backward writes dk,
    dv and the max-pool scatter of dq into ONE dqkv buffer (separate select / slice inputs made
    autograd zero-fill a qkv-sized buffer per slice and add them)."""

    @staticmethod
    def forward(ctx, qkv, nh):
        B, H, W, d3 = qkv.shape
        d = d3 // 3
        hd = d // nh
        q = ops.maxpool2(qkv[..., :d]).view(B, (H // 2) * (W // 2), nh, hd)
        qkv5 = qkv.view(B, H * W, 3, nh, hd)
        o = torch.empty(q.shape, device=qkv.device, dtype=qkv.dtype)
        lse = torch.empty(B, nh, q.shape[1], device=qkv.device, dtype=torch.float32)
        scale = 1.0 / math.sqrt(hd)
        ops.attn_fwd(q, qkv5[:, :, 1], qkv5[:, :, 2], o, lse, scale)
        ctx.nh, ctx.scale = nh, scale
        ctx.save_for_backward(qkv, q, o, lse)
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, q, o, lse = ctx.saved_tensors
        B, H, W, d3 = qkv.shape
        d = d3 // 3
        qkv5 = qkv.view(B, H * W, 3, ctx.nh, d // ctx.nh)
        dqkv = torch.empty_like(qkv)
        dqkv5 = dqkv.view(qkv5.shape)
        dq = torch.empty_like(q)
        ops.attn_bwd(q, qkv5[:, :, 1], qkv5[:, :, 2], o, do.contiguous(), lse, dq, dqkv5[:, :, 1], dqkv5[:, :, 2],
                     ctx.scale)
        ops.maxpool2_bwd(qkv[..., :d], dq.view(B, H // 2, W // 2, d), dqkv[..., :d])
        return dqkv, None


def pooled_qkv_attention(qkv, num_heads):
    """attention of the 2x2-max-pooled q third of a fused [B, H, W, 3d] projection against its full
    k / v (Hiera's stage-transition blocks) -> [B, H/2 * W/2, heads, d / heads]"""
    return _PoolQKVAttention.apply(qkv, num_heads)


def qkv_attention(qkv, scale=None, p_drop=0.0, rope=None):
    """softmax(scale q k^T) v with q, k, v = qkv[:, :, 0/1/2] ([B, L, 3, H, d]); rope = (cos, sin,
    period) rotates q and k (every row) first."""
    if scale is None:
        scale = 1.0 / math.sqrt(qkv.shape[-1])
    T = _ft.active()
    if T is not None:
        return _ft.qkv_attention(T, qkv, float(scale), float(p_drop), rope)
    return _QKVAttention.apply(qkv, float(scale), float(p_drop), rope)


# ------------------------------------------------------------------ RoPE
class _Rope(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, nrot, cos, sin, period):
        # x [Bt, L, D]; rotates rows < nrot, copies the rest
        y = torch.empty_like(x)
        if nrot < x.shape[1]:
            y[:, nrot:].copy_(x[:, nrot:])
        ops.rope(x, y, nrot, cos, sin, period)
        ctx.nrot, ctx.period = nrot, period
        ctx.save_for_backward(cos, sin)
        return y

    @staticmethod
    def backward(ctx, dy):
        cos, sin = ctx.saved_tensors
        dy = dy.contiguous()
        dx = torch.empty_like(dy)
        if ctx.nrot < dy.shape[1]:
            dx[:, ctx.nrot:].copy_(dy[:, ctx.nrot:])
        ops.rope(dy, dx, ctx.nrot, cos, sin, ctx.period, inverse=True)
        return dx, None, None, None, None


def rope(x, nrot, cos, sin, period):
    T = _ft.active()
    if T is not None:
        return _ft.rope(T, x, int(nrot), cos, sin, int(period))
    return _Rope.apply(x.contiguous(), int(nrot), cos, sin, int(period))


# ------------------------------------------------------ elementwise / misc
class _Add(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b, alpha, beta):
        ctx.alpha, ctx.beta = alpha, beta
        return ops.add(a.contiguous(), b.contiguous(), alpha=alpha, beta=beta)

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        da = g if ctx.alpha == 1.0 else ops.add(g, None, alpha=ctx.alpha)
        db = g if ctx.beta == 1.0 else ops.add(g, None, alpha=ctx.beta)
        return (da if ctx.needs_input_grad[0] else None), (db if ctx.needs_input_grad[1] else None), None, None


def add(a, b, alpha=1.0, beta=1.0):
    T = _ft.active()
    if T is not None:
        return _ft.add(T, a, b, float(alpha), float(beta))
    return _Add.apply(a, b, float(alpha), float(beta))


class _AddBcast(torch.autograd.Function):
    """out[o, ...] = alpha*a[o, ...] + beta*b[...]   (b broadcast over the leading dim)."""

    @staticmethod
    def forward(ctx, a, b, alpha, beta, shape, bparam):
        out = ops.add_bcast(a.contiguous() if a is not None else None, b.contiguous(), alpha=alpha, beta=beta,
                            shape=shape if a is None else None)
        ctx.alpha, ctx.beta, ctx.bshape, ctx.bparam = alpha, beta, b.shape, bparam
        ctx.has_a = a is not None
        return out

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        da = None
        if ctx.has_a and ctx.needs_input_grad[0]:
            da = g if ctx.alpha == 1.0 else ops.add(g, None, alpha=ctx.alpha)
        db = None
        inner = math.prod(ctx.bshape)
        O = g.numel() // inner
        if ctx.bparam is not None:
            gb = _grad_of(ctx.bparam)
            if gb is not None:
                if ctx.beta == 1.0:
                    ops.colsum(g.view(O, inner), gb.view(-1), accumulate=True)
                else:
                    tmp = torch.zeros(inner, device=g.device, dtype=torch.float32)
                    ops.colsum(g.view(O, inner), tmp)
                    ops.add(gb.view(-1), tmp, beta=ctx.beta, out=gb.view(-1))
        elif ctx.needs_input_grad[1]:
            db = torch.empty(ctx.bshape, device=g.device, dtype=g.dtype)
            ops.sum_outer(g.view(O, inner), db.view(-1))
            if ctx.beta != 1.0:
                db = ops.add(db, None, alpha=ctx.beta)
        return da, db, None, None, None, None


def add_bcast(a, b, alpha=1.0, beta=1.0, shape=None, bparam=None):
    """a + beta*b with b broadcast over leading dims.  If `bparam` (a Parameter) is given,
    b is its compute copy and its gradient goes to the arena."""
    T = _ft.active()
    if T is not None:
        return _ft.add_bcast(T, a, b, float(alpha), float(beta), shape, bparam)
    return _AddBcast.apply(a, b, float(alpha), float(beta), shape, bparam)


class _Act(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, act):
        ctx.act = act
        ctx.save_for_backward(x)
        return ops.act_fwd(x.contiguous(), act)

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        return ops.act_bwd(x, g.contiguous(), ctx.act), None


def act(x, a):
    T = _ft.active()
    if T is not None:
        return _ft.act(T, x, a)
    return _Act.apply(x, a)


class _Dropout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p):
        ctx.p = p
        ctx.seed = next_seed()
        return ops.dropout(x.contiguous(), p, ctx.seed)

    @staticmethod
    def backward(ctx, g):
        return ops.dropout(g.contiguous(), ctx.p, ctx.seed), None


def dropout(x, p, training=True):
    if not training or p <= 0.0:
        return x
    return _Dropout.apply(x, float(p))


class _MaxPool2(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.save_for_backward(x)
        return ops.maxpool2(x)

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        dx = torch.empty(x.shape, device=x.device, dtype=x.dtype)
        ops.maxpool2_bwd(x, g.contiguous(), dx)
        return dx


def maxpool2(x):
    """2x2 max-pool of NHWC x (pixel stride may exceed C: reads q out of a fused qkv)."""
    return _MaxPool2.apply(x)


class _WindowPartition(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, ws):
        ctx.ws = ws
        ctx.shape = x.shape
        return ops.window_partition(x.contiguous(), ws)

    @staticmethod
    def backward(ctx, g):
        B, H, W, C = ctx.shape
        return ops.window_unpartition(g.contiguous(), ctx.ws, B, H, W), None


class _WindowUnpartition(torch.autograd.Function):
    @staticmethod
    def forward(ctx, win, ws, B, H, W):
        ctx.ws, ctx.BHW = ws, (B, H, W)
        return ops.window_unpartition(win.contiguous(), ws, B, H, W)

    @staticmethod
    def backward(ctx, g):
        return ops.window_partition(g.contiguous(), ctx.ws), None, None, None, None


class _WindowPad(torch.autograd.Function):
    """partition(linear(x)) with the padded positions = linear's bias (= linear(partition(x)) of the
    zero-padded partition, hieradet.py:146): the linear ran over the real tokens only.  Backward: the
    real rows' gradient by unpartition; the padded rows' column sums go to the linear's bias
    gradient (the arena; accumulating, like every weight-gradient write of the step)."""

    @staticmethod
    def forward(ctx, y, ws, mod):
        ctx.ws, ctx.shape, ctx.mod = ws, y.shape, mod
        return ops.window_pad(y.contiguous(), ws, mod.compute_bias())

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        B, H, W, C = ctx.shape
        gb = ctx.mod.grad_views()[1]
        if gb is not None:
            ops.window_pad_colsum(g, ctx.ws, B, H, W, gb.view(-1))
        return ops.window_unpartition(g, ctx.ws, B, H, W), None, None


def window_pad(y, ws, mod):
    """partition of linear `mod`'s output y [B, H, W, C] into ws x ws windows, padded positions = the
    bias (what `mod` gives for a zero-padded input row)"""
    assert mod.compute_bias() is not None
    return _WindowPad.apply(y, int(ws), mod)


def window_partition(x, ws):
    return _WindowPartition.apply(x, int(ws))


def window_unpartition(win, ws, B, H, W):
    return _WindowUnpartition.apply(win, int(ws), int(B), int(H), int(W))


class _Up2Add(torch.autograd.Function):
    @staticmethod
    def forward(ctx, lat, prev):
        return ops.up2_add(lat.contiguous(), prev.contiguous())

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        B, H, W, C = g.shape
        dprev = torch.empty(B, H // 2, W // 2, C, device=g.device, dtype=g.dtype)
        ops.pool2_sum(g, dprev)
        return g, dprev


def up2_add(lat, prev):
    """FPN top-down: lat + nearest-x2(prev), NHWC"""
    return _Up2Add.apply(lat, prev)


class _Bilinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, ho, wo):
        ctx.hw = x.shape[-2:]
        return ops.bilinear(x.contiguous(), ho, wo)

    @staticmethod
    def backward(ctx, g):
        return ops.bilinear_bwd(g.contiguous(), ctx.hw[0], ctx.hw[1]), None, None


def bilinear(x, ho, wo):
    """[N, hi, wi] f32 -> [N, ho, wo] bilinear (align_corners=False)"""
    T = _ft.active()
    if T is not None:
        return _ft.bilinear(T, x, int(ho), int(wo))
    return _Bilinear.apply(x, int(ho), int(wo))


class _RowGate(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gate, fill):
        ctx.save_for_backward(gate)
        return ops.row_gate(x.contiguous(), gate, fill)

    @staticmethod
    def backward(ctx, g):
        (gate,) = ctx.saved_tensors
        return ops.row_gate(g.contiguous(), gate, 0.0, backward=True), None, None


def row_gate(x, gate, fill):
    """x[r] if gate[r] > 0 else fill (gate is a non-differentiable f32 [R])"""
    T = _ft.active()
    if T is not None:
        return _ft.row_gate(T, x, gate, float(fill))
    return _RowGate.apply(x, gate, float(fill))


def cast_gate(x, dtype, gate, fill):
    """row_gate(cast(x, dtype), gate, fill); on the frame tape one op and one launch"""
    T = _ft.active()
    if T is not None and x.dtype != dtype and os.environ.get("S2H_CAST_GATE", "1") != "0" \
            and gate.dtype == torch.float32 and gate.is_contiguous() and gate.numel() == x.shape[0]:
        return _ft.cast_gate(T, x, dtype, gate, float(fill))
    return row_gate(cast(x, dtype), gate, fill)


class _Cast(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dtype):
        ctx.dtype = x.dtype
        return ops.cast(x.contiguous(), dtype)

    @staticmethod
    def backward(ctx, g):
        return ops.cast(g.contiguous(), ctx.dtype), None


def cast(x, dtype):
    if x.dtype == dtype:
        return x
    T = _ft.active()
    if T is not None:
        return _ft.cast(T, x, dtype)
    return _Cast.apply(x, dtype)


class _SumOuter(torch.autograd.Function):
    """x [1, ...] broadcast to [O, ...]: forward copies, backward sums over O."""

    @staticmethod
    def forward(ctx, x, O):
        ctx.O = O
        out = ops.add_bcast(None, x.contiguous(), shape=(O, *x.shape[1:]))
        return out

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        d = torch.empty((1, *g.shape[1:]), device=g.device, dtype=g.dtype)
        ops.sum_outer(g, d.view(-1))
        return d, None


def expand_batch(x, O):
    """[1, ...] -> [O, ...] materialised broadcast (grad = sum over O)"""
    T = _ft.active()
    if T is not None:
        return _ft.expand_batch(T, x, int(O))
    return _SumOuter.apply(x, int(O))


class _SelectToken(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, i):
        ctx.shape, ctx.i = x.shape, i
        return x[:, i].contiguous()

    @staticmethod
    def backward(ctx, g):
        d = torch.zeros(ctx.shape, device=g.device, dtype=g.dtype)
        d[:, ctx.i].copy_(g)
        return d, None


def select_token(x, i):
    """x [B, N, C] -> x[:, i] as a contiguous [B, C] (the decoder's output-token reads)"""
    T = _ft.active()
    if T is not None:
        return _ft.select_token(T, x, int(i))
    return _SelectToken.apply(x, int(i))


def select_tokens(x, idxs):
    """[select_token(x, i) for i in idxs]; on the frame tape one op and one copy launch"""
    T = _ft.active()
    if T is not None and _ft.select_tokens_ok(x):
        return _ft.select_tokens(T, x, [int(i) for i in idxs])
    return [select_token(x, i) for i in idxs]
