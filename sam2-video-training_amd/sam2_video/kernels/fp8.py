"""MX-fp8 compute mode (BASELINE config 5: `compute_dtype="fp8"`, Lightning precision "fp8").

Recipe: among the projection and FFN Linear layers of the image encoder trunk and the memory
attention, the widening GEMMs run on MX-fp8 operands (OCP MXFP8-E4M3, 32-element blocks along the
reduction dimension, csrc/gemm_mx8.hip): the forward of layers with in < out (Hiera qkv and MLP
fc1, the FFN's linear1): Y = Q(X) Q(W)^T, and the input gradient of layers with out < in (MLP
fc2, linear2): dX = Q(dY) Q(W^T)^T -- see `_pays`.  The weight gradients stay
bf16 (dW = dY^T X over 10^4-10^5 token rows from the saved bf16 activations, fp32 accumulate),
as do activations between kernels, attention, norms, losses, the fp32 master weights and AdamW.

Weight operands are quantised from the bf16 shadow once per forward (`new_step`, called at the
top of SAM2Model.forward, so a captured step graph re-quantises on every replay after AdamW
moved the weights): the forward operand Q(W) [N, Kp] on first forward use, the dgrad operand
Q(W^T) [K, Np] on first backward use.  Activation and gradient operands are quantised right
before each GEMM (one bf16 read, one fp8 write).
"""
from __future__ import annotations

import torch

from . import ops

_STATE = {"gen": 0}

# module name prefixes whose Linear layers take the MX-fp8 path.  The mask decoder's two-way
# transformer stays bf16: a negligible share of the flops (<= 8 tokens x 4096 keys per object)
# and the most quantisation-sensitive layers of the step (tools/fp8_drift.py at B+ 256^2 against
# the fp32 mode: two-way in fp8 -> mask IoU 0.95-0.97, memory attention -> 0.988-0.995,
# trunk -> 0.954-0.963; bf16 everywhere -> 0.992-0.995)
FP8_PREFIXES = ("image_encoder.trunk.", "memory_attention.")
MIN_IN_FEATURES = 128  # narrower inputs would be mostly padding in a 128-deep MX step
# input-gradient GEMMs on MX-fp8 too (False: forward only, dgrad in bf16)
DGRAD = {"on": True}


def new_step():
    _STATE["gen"] += 1


def mark_modules(model):
    """flag the fp8-eligible Linear layers of `model` (SAM2Model.load with compute_dtype fp8)"""
    from ..model.modeling.layers import Linear
    n = 0
    for name, m in model.named_modules():
        if type(m) is Linear and name.startswith(FP8_PREFIXES) and m.in_features >= MIN_IN_FEATURES \
                and m.out_features >= 64:
            m._s2h_fp8 = True
            n += 1
    return n


def _eligible(mod):
    f = getattr(mod, "_s2h_fp8", None)
    if f is None:
        members = getattr(mod, "members", None)  # FusedLinear: all members flagged
        f = bool(members) and all(getattr(m, "_s2h_fp8", False) for m in members)
    return f


class _Entry:
    __slots__ = ("fwd", "t", "gen_f", "gen_t")

    def __init__(self):
        self.fwd = self.t = None
        self.gen_f = self.gen_t = -1


def _entry(mod):
    e = getattr(mod, "_s2h_fp8_entry", None)
    if e is None:
        e = _Entry()
        mod._s2h_fp8_entry = e
    return e


def weight(mod):
    """MX-fp8 forward operand Q(W) [N, Kp] of `mod` for this step, or None (bf16 path)"""
    if not _eligible(mod):
        return None
    e = _entry(mod)
    if e.gen_f != _STATE["gen"]:
        w = mod.compute_weight()
        if e.fwd is None:
            e.fwd = ops.mx8_empty(w.shape[0], w.shape[1], w.device)
        ops.mx8_quant(w, out=e.fwd)
        e.gen_f = _STATE["gen"]
    return e.fwd


def weight_t(mod):
    """MX-fp8 dgrad operand Q(W^T) [K, Np] of `mod` for this step, or None"""
    if not _eligible(mod):
        return None
    e = _entry(mod)
    if e.gen_t != _STATE["gen"]:
        w = mod.compute_weight()
        if e.t is None:
            e.t = ops.mx8_empty(w.shape[1], w.shape[0], w.device)
        ops.mx8_quant(w, out=e.t, transpose=True)
        e.gen_t = _STATE["gen"]
    return e.t


def _pays(k_reduce, n_out):
    """MX-fp8 only where the quantiser pass over the activation operand ([rows, k_reduce]: one
    bf16 read + one fp8 write) is cheaper than what the faster GEMM saves.  The step's GEMMs are
    short-K and store-bound, so the saving is a fraction of the OUTPUT traffic ([rows, n_out]):
    widening layers (k < n: Hiera qkv / MLP fc1, memory-attention FFN linear1, and the dgrads of
    the narrowing layers) pay; K = N projections break even and narrowing layers (MLP fc2, FFN
    linear2 forward over a 4x-wide input) lose -- rocprofv3 of config 5 with every projection on
    MX-fp8: the quantiser passes took 8.5 ms per step, more than the MX GEMMs saved."""
    return k_reduce < n_out


def linear(x, mod, w, bias, **kw):
    """forward GEMM of a Linear: MX-fp8 when `mod` is eligible (and it pays), else the bf16 kernel"""
    w8 = weight(mod) if x.dtype != torch.float32 and _pays(w.shape[1], w.shape[0]) else None
    if w8 is not None:
        return ops.linear_mx8(x, w8, bias, **kw)
    return ops.linear(x, w, bias, **kw)


def linear_rope(x, mod, w, bias, rope, out=None):
    """forward GEMM of a Linear whose output is rotated by RoPE (ops.rope_blocks layout): MX-fp8
    GEMM + in-place rotation when `mod` is eligible, else the bf16 GEMM with the rotation fused"""
    w8 = weight(mod) if x.dtype != torch.float32 and _pays(w.shape[1], w.shape[0]) else None
    if w8 is not None:
        out = ops.linear_mx8(x, w8, bias, out=out)
        ops.rope_blocks(out.view(-1, out.shape[-1]), rope)
        return out
    return ops.linear_rope(x, w, bias, rope, out=out)


def dgrad_on_mx8(dy, mod):
    """linear_dgrad of `mod` runs on MX-fp8 operands"""
    return dy.dtype != torch.float32 and DGRAD["on"] and _eligible(mod) and _pays(mod.out_features, mod.in_features)


def linear_dgrad(dy, mod, **kw):
    """input-gradient GEMM of a Linear: MX-fp8 when `mod` is eligible (and it pays), else the bf16 kernel"""
    wt8 = weight_t(mod) if dgrad_on_mx8(dy, mod) else None
    if wt8 is not None:
        return ops.linear_dgrad_mx8(dy, wt8, **kw)
    return ops.linear_dgrad(dy, mod.compute_weight(), **kw)
