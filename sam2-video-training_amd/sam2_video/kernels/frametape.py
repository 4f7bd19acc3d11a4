"""Frame-batched backward of the tracking loop.

The tracking loop (reference sam2model.py:266-401) is sequential in the forward -- frame t reads
the memory bank written by frames < t -- but its backward is not: the bank entries and object
pointers are detached (sam2model.py:340-358), so every frame's graph ends at the bank and the
frames' backwards are independent.  Running them one frame at a time (autograd) leaves every
GEMM at 13 objects x 1024 tokens and every flash-attention backward at 13 batches: latency-bound
launches far below the MFMA roofline.

A FrameTape records the per-frame ops of one program (the memory attention of frames 1..T-1, or
the SAM heads of frames 0..T-1).  Every frame runs the SAME op sequence; op k's outputs at frame
f are written straight into slot f of a [F, ...] buffer (or, for the memory-bank-sized tensors
whose row count grows with the frame, into frame f's rows of a packed buffer), so everything the
backward needs is already stacked.  The backward walks the ops once in reverse and runs each op
over all frames: one dgrad GEMM, one weight-gradient GEMM, one LayerNorm backward, one flash
backward (s2h_flash_bwd_frames, packed per-frame K/V) per op instead of F of each.

Dropout stays mask-identical to the per-frame forward: a dropout site draws one seed and frame
f's launch offsets its element indices by the elements of frames < f (the kernels' idx0), so the
stacked backward regenerates exactly the forward's masks.

While a tape is recording, the sam2_video.kernels.functional ops dispatch here (`active()`); the
module code is shared with the autograd path.  Test infrastructure compares both paths
(tests/test_frametape_gpu.py).
"""
from __future__ import annotations

import collections
import math
import os
from typing import Dict, List, Optional

import torch

from . import fp8 as _fp8
from . import ops

_ACTIVE: List[Optional["FrameTape"]] = [None]


def active() -> Optional["FrameTape"]:
    """the recording tape, when the op runs with autograd enabled (no_grad regions of the
    tracking loop -- object pointers, memory encoder -- run the plain kernels)"""
    t = _ACTIVE[0]
    return t if (t is not None and torch.is_grad_enabled()) else None


class recording:
    """context: the FN ops record into `tape` for its current frame"""

    def __init__(self, tape):
        self.tape = tape

    def __enter__(self):
        self.prev = _ACTIVE[0]
        _ACTIVE[0] = self.tape
        return self.tape

    def __exit__(self, *exc):
        _ACTIVE[0] = self.prev


def _grad_of(p):
    return getattr(p, "_s2h_grad", None) if p is not None and p.requires_grad else None


# ------------------------------------------------------------------------- storage
class Store:
    """A value's frame-stacked storage: uniform [F, *shape] or packed (frame f's rows at
    offsets[f] of a flat [total] buffer; the per-frame element count scales with the frame's
    memory rows)."""

    def __init__(self, tape, shape, dtype, scale=None, alias=None):
        self.shape0 = tuple(shape)
        self.dtype = dtype
        F = tape.F
        n0 = math.prod(shape)
        self.aliased = alias is not None
        if alias is not None:  # uniform storage the caller already holds
            assert scale is None and alias.numel() == F * n0 and alias.dtype == dtype
            self.numels = [n0] * F
            self.buf = alias
        elif scale is None:  # uniform
            self.numels = [n0] * F
            self.buf = torch.empty(F * n0, device=tape.device, dtype=dtype)
        else:  # element count of frame f = n0 * scale[f] / scale[0]
            assert all(n0 * s % scale[0] == 0 for s in scale)
            self.numels = [n0 * s // scale[0] for s in scale]
            self.buf = torch.empty(sum(self.numels), device=tape.device, dtype=dtype)
        self.offsets = [0]
        for n in self.numels[:-1]:
            self.offsets.append(self.offsets[-1] + n)
        self.uniform = scale is None
        self.scale = scale
        if scale is not None:  # the varying dim: the one of size scale[0] (memory rows), unique
            hits = [i for i, d in enumerate(self.shape0) if d == scale[0]]
            assert len(hits) == 1, f"ambiguous memory-row dim in {self.shape0} (rows {scale[0]})"
            self.vdim = hits[0]

    def frame_shape(self, f):
        if self.uniform:
            return self.shape0
        sh = list(self.shape0)
        sh[self.vdim] = self.scale[f]
        return tuple(sh)

    def frame(self, f):
        return self.buf[self.offsets[f]:self.offsets[f] + self.numels[f]].view(self.frame_shape(f))

    def stacked(self, lead=None):
        """uniform: [F, *shape] (or [F * shape[0], *shape[1:]] with lead='merge'); packed: flat"""
        if not self.uniform:
            return self.buf
        F = len(self.numels)
        if lead == "merge":
            return self.buf.view(F * self.shape0[0], *self.shape0[1:])
        return self.buf.view(F, *self.shape0)


def _alias_rows(stacked, F, t):
    """flat view of frames [first, first + F) of a frame-stacked tensor, when contiguous"""
    if stacked is None:
        return None
    src, first = stacked
    if src.dtype != t.dtype or not src.is_contiguous() or first + F > src.shape[0]:
        return None
    if src[first].numel() != t.numel():
        return None
    return src[first:first + F].reshape(-1)


class FlatStore:
    """a saved per-frame buffer of explicit per-frame element counts (flat, frame f from offsets[f])"""

    def __init__(self, tape, numels, dtype):
        self.numels = [int(n) for n in numels]
        self.offsets = [0]
        for n in self.numels[:-1]:
            self.offsets.append(self.offsets[-1] + n)
        self.buf = torch.empty(sum(self.numels), device=tape.device, dtype=dtype)

    def frame(self, f):
        return self.buf[self.offsets[f]:self.offsets[f] + self.numels[f]]


class Op:
    __slots__ = ("kind", "idx", "ins", "outs", "attrs", "fattrs", "saved", "needs", "bw")

    def __init__(self, kind, ins, outs, attrs, bw):
        self.kind = kind
        self.idx = -1
        self.ins = ins      # input value ids (None = constant / param-only)
        self.outs = outs    # output value ids
        self.attrs = attrs  # frame-invariant attributes
        self.fattrs = {}    # per-frame attribute lists
        self.saved = {}     # name -> value id / Store / per-frame list
        self.needs = None
        self.bw = bw


class FrameTape:
    def __init__(self, nframes: int, device, mem_rows: Optional[List[int]] = None, name: str = ""):
        self.F = int(nframes)
        self.device = device
        self.name = name
        self.mem_rows = list(mem_rows) if mem_rows is not None else None
        self.ops: List[Op] = []
        self.f = -1
        self.k = 0
        self.stores: Dict[object, Store] = {}   # value id -> Store
        self.requires: Dict[object, bool] = {}  # value id -> needs grad
        self.ptr2vid: Dict[int, object] = {}    # current frame: data_ptr -> value id
        self.inputs: Dict[str, object] = {}     # declared grad-carrying frame inputs
        self._seeds: Dict[int, int] = {}

    # ------------------------------------------------------------ frames
    def begin_frame(self):
        self.f += 1
        assert self.f < self.F, f"tape {self.name}: more frames than declared ({self.F})"
        self.k = 0
        self.ptr2vid = {}

    def end_frame(self):
        assert self.k == len(self.ops), f"tape {self.name}: frame {self.f} ran {self.k} ops, frame 0 {len(self.ops)}"

    # ------------------------------------------------------------ values
    def _register(self, vid, t):
        self.ptr2vid[t.data_ptr()] = vid

    def vid(self, t):
        """value id of a tensor produced by this frame's ops (None = constant)"""
        if t is None:
            return None
        v = self.ptr2vid.get(t.data_ptr())
        if v is None and self.f == 0:
            self._check_const(t)
        return v

    def _check_const(self, t):
        # a constant must not alias tape storage (a view the tape did not record)
        p0, p1 = t.data_ptr(), t.data_ptr() + t.numel() * t.element_size()
        for st in self.stores.values():
            b0 = st.buf.data_ptr()
            b1 = b0 + st.buf.numel() * st.buf.element_size()
            if p0 < b1 and b0 < p1:
                raise RuntimeError(f"tape {self.name}: tensor aliases tape storage but is not a recorded value "
                                   f"(slice / copy outside the FN ops?)")

    def input(self, name, t, requires_grad=True, stacked=None):
        """declare a grad-carrying per-frame input (e.g. the backbone feature of this frame): its
        frame values are stacked (copied) so the backward can return [F, ...] gradients.
        stacked = (tensor, first): the caller's values already ARE frame-stacked -- this tape's
        frame f is tensor[first + f] (contiguous) -- and the store aliases them (no copy)."""
        vid = ("in", name)
        if self.f == 0:
            st = Store(self, t.shape, t.dtype, alias=_alias_rows(stacked, self.F, t))
            self.stores[vid] = st
            self.requires[vid] = requires_grad
            self.inputs[name] = vid
        st = self.stores[vid]
        slot = st.frame(self.f)
        if st.aliased:
            assert slot.data_ptr() == t.data_ptr(), f"tape {self.name}: input {name} is not the stacked frame"
        else:
            slot.copy_(t.detach())
        self._register(vid, slot)
        return slot

    def varlen_slot(self, name, shape, dtype):
        """a packed per-frame buffer for a constant whose row count follows the memory rows (the
        assembled memory bank): written by the caller, read by the ops as a value"""
        vid = ("const", name)
        if self.f == 0:
            self.stores[vid] = Store(self, shape, dtype, scale=self.mem_rows)
            self.requires[vid] = False
        slot = self.stores[vid].frame(self.f)
        assert tuple(slot.shape) == tuple(shape), (slot.shape, shape)
        self._register(vid, slot)
        return slot

    def _varlen_scale(self, *ts):
        for t in ts:
            v = self.vid(t) if t is not None else None
            if v is not None and not self.stores[v].uniform:
                return self.stores[v].scale
        return None

    def _out(self, j, shape, dtype, scale=None):
        """output j of the current op at this frame (allocated on frame 0)"""
        vid = (self.k, j)
        if self.f == 0:
            self.stores[vid] = Store(self, shape, dtype, scale=scale)
        slot = self.stores[vid].frame(self.f)
        assert tuple(slot.shape) == tuple(shape), (self.name, self.k, slot.shape, shape)
        self._register(vid, slot)
        return vid, slot

    def _aux(self, name, shape, dtype, scale=None):
        """frame-stacked saved buffer of the current op (not a value)"""
        key = ("aux", self.k, name)
        if self.f == 0:
            self.stores[key] = Store(self, shape, dtype, scale=scale)
        return self.stores[key].frame(self.f)

    def _aux_flat(self, name, numels, dtype):
        """frame-stacked saved flat buffer of the current op with per-frame sizes `numels` (all frames)"""
        key = ("aux", self.k, name)
        if self.f == 0:
            self.stores[key] = FlatStore(self, numels, dtype)
        return self.stores[key].frame(self.f)

    def _keep_bits(self, q, Lk, kvid, p_drop):
        """dropout keep bitmap slot of this frame's attention (None: the kernels re-hash), sized for
        every frame's key count (packed per frame when the key value `kvid` follows the memory rows)"""
        if not ops.keep_bits_ok(q, p_drop):
            return None
        B, Lq, H, _ = q.shape
        st = self.stores.get(kvid) if kvid is not None else None
        scale = st.scale if st is not None and not st.uniform else None
        lks = [Lk] * self.F if scale is None else [Lk * sc // scale[self.f] for sc in scale]
        return self._aux_flat("keep", [ops.keep_words(B, H, Lq, lk) for lk in lks], torch.int32)

    def _begin(self, kind, ins, bw, attrs=None):
        """start op `kind` at the current frame; returns (op, is_first_frame)"""
        if self.f == 0:
            op = Op(kind, [self.vid(t) if torch.is_tensor(t) else None for t in ins], [], attrs or {}, bw)
            op.needs = [v is not None and self.requires.get(v, False) for v in op.ins]
            op.idx = len(self.ops)
            self.ops.append(op)
            return op, True
        op = self.ops[self.k]
        assert op.kind == kind, f"tape {self.name}: frame {self.f} op {self.k} is {kind}, frame 0 had {op.kind}"
        got = [self.vid(t) if torch.is_tensor(t) else None for t in ins]
        assert got == op.ins, f"tape {self.name}: op {self.k} ({kind}) inputs differ between frames"
        return op, False

    def _finish(self, op, outs_vids, req):
        if self.f == 0:
            op.outs = outs_vids
            for v in outs_vids:
                self.requires[v] = req
        self.k += 1

    def _seed(self):
        from .functional import next_seed
        if self.f == 0:
            s = next_seed()
            self._seeds[self.k] = s
            return s
        return self._seeds[self.k]

    def _fattr(self, op, name, value):
        lst = op.fattrs.setdefault(name, [])
        assert len(lst) == self.f
        lst.append(value)

    def _idx0(self, op, numel):
        """dropout element offset of this frame: elements of all earlier frames of the site"""
        lst = op.fattrs.setdefault("idx0", [])
        n = op.fattrs.setdefault("numel", [])
        assert len(lst) == self.f
        lst.append(0 if self.f == 0 else lst[-1] + n[-1])
        n.append(numel)
        return lst[-1]

    def _req(self, op, params=()):
        return any(op.needs) or any(p is not None and p.requires_grad and _grad_of(p) is not None for p in params)

    # ------------------------------------------------------------ backward
    def backward(self, out_grads: Dict[object, torch.Tensor]):
        """out_grads: value id -> stacked gradient.  Returns {input name: stacked gradient}."""
        G = dict(out_grads)
        owned = set()
        self.producer = {v: op for op in self.ops for v in op.outs}
        self.nuse = collections.Counter(v for op in self.ops for v in op.ins if v is not None)
        self.first_use = {}  # value id -> index of the first op reading it
        for op in self.ops:
            for v in op.ins:
                if v is not None and v not in self.first_use:
                    self.first_use[v] = op.idx
        self.premasked = set()
        self.prefused_dx = {}  # linear op index -> its input gradient, computed by its consumer (FFN fusion)
        self.derotated = set()  # linear-with-RoPE outputs whose consumer returned the un-rotated gradient
        self.derotated_cols = {}  # ... whose consumer un-rotated the gradient's columns < the value
        self.seeded = set(out_grads)

        def acc(vid, g):
            if vid is None or g is None:
                return
            if vid not in G:
                G[vid] = g
                return
            if vid in owned:
                ops.add(G[vid], g, out=G[vid])
            else:
                G[vid] = ops.add(G[vid], g)
                owned.add(vid)

        self.grads, self.acc = G, acc  # for ops whose backward finishes their producer's (_ln_dgrad_fused)
        self.owned = owned  # gradients this backward allocated (safe to add into in place)
        self.side = ops.SideWork()  # the Linear weight gradients' stream (joined before returning)
        for k in range(len(self.ops) - 1, -1, -1):
            op = self.ops[k]
            gys = [G.pop(v, None) for v in op.outs]
            if all(g is None for g in gys):
                continue
            gins = op.bw(self, op, gys)
            for v, need, g in zip(op.ins, op.needs, gins):
                if need:
                    acc(v, g)
        self.side.join()
        self.grads = self.acc = self.owned = None
        return {name: G.get(vid) for name, vid in self.inputs.items()}

    def out_vid(self, t):
        """value id of a recorded output (to seed the backward)"""
        return self.ptr2vid[t.data_ptr()]

    def st(self, vid) -> Store:
        return self.stores[vid]


# =============================================================================== ops
# Each op: forward at the current frame (writes slots) + batched backward over all frames.

def _flat(st: Store, width):
    """stacked storage as [rows, width]"""
    return st.buf.view(-1, width)


def _empty_like_store(tape, st: Store, dtype=None):
    return torch.empty(st.buf.numel(), device=st.buf.device, dtype=dtype or st.dtype)


# ---------------------------------------------------------------- linear
def linear(tape: FrameTape, x, mod, act=None, residual=None, drop_p=0.0, rope=None, _compute=True):
    """_compute=False records the op and returns its output slot without launching (a fused kernel
    writes it: dec_self / dec_post / dec_final)"""
    x = x if x.is_contiguous() else x.contiguous()
    # ReLU without residual: the backward masks with the output (> 0 exactly where the
    # pre-activation was positive and the element kept), so no pre-activation is stored
    relu_out = act == "relu" and residual is None
    op, first = tape._begin("linear", [x, residual], _linear_bw,
                            {"mod": mod, "act": act, "p": float(drop_p), "relu_out": relu_out,
                             "rope": rope is not None})
    if first and tape.vid(x) is None:
        raise RuntimeError("tape linear: input must be a recorded value or declared input")
    w = mod.compute_weight()
    b = mod.compute_bias()
    N = w.shape[0]
    scale = tape._varlen_scale(x)
    shape = (*x.shape[:-1], N)
    vid, out = tape._out(0, shape, x.dtype, scale)
    pre = tape._aux("pre", shape, x.dtype, scale) if act and not relu_out else None
    seed = tape._seed() if drop_p > 0 else 0
    idx0 = tape._idx0(op, out.numel())
    if not _compute:
        assert rope is None and pre is None and drop_p == 0
    elif rope is not None:  # RoPE of the output in the GEMM epilogue; per-frame (L, nrot) for the backward
        assert act is None and residual is None and drop_p == 0
        _fp8.linear_rope(x, mod, w, b, rope, out=out)
        tape._fattr(op, "rope", rope)
    else:
        _fp8.linear(x, mod, w, b, act=act, out=out, pre=pre, residual=residual, drop_p=drop_p, seed=seed,
                    drop_idx0=idx0)
    if first:
        op.attrs["seed"] = seed
        op.attrs["K"] = x.shape[-1]
    tape._finish(op, [vid], tape._req(op, (mod.weight, mod.bias)))
    return out


def ffn_fwd_ok(x, mod1, mod2):
    """ops.ffn_fwd applies to linear2(drop(relu(linear1(x)))) on the tape (bf16, not MX-fp8)"""
    if _fp8._eligible(mod1) or _fp8._eligible(mod2):
        return False
    x2 = x.reshape(-1, x.shape[-1]) if x.is_contiguous() else None
    return x2 is not None and ops.ffn_fwd_ok(x2, mod1.compute_weight(), mod1.compute_bias(), mod2.compute_weight(),
                                            mod2.compute_bias())


def ffn(tape: FrameTape, x, mod1, mod2, drop_p=0.0):
    """linear(x, mod1, relu, drop_p) -> linear(., mod2, drop_p) (memory_attention.py:97), recorded as
    exactly those two tape ops -- same op records, seeds and dropout element offsets as two `linear`
    calls, so the backward is theirs (the ReLU linear's consumer runs ops.ffn_bwd_dgrad) -- but
    computed by ONE ops.ffn_fwd launch: hid is written once for the backward and never re-read here."""
    w1, b1, w2, b2 = mod1.compute_weight(), mod1.compute_bias(), mod2.compute_weight(), mod2.compute_bias()
    H, C = w1.shape
    N = w2.shape[0]
    scale = tape._varlen_scale(x)
    op1, first1 = tape._begin("linear", [x, None], _linear_bw,
                              {"mod": mod1, "act": "relu", "p": float(drop_p), "relu_out": True, "rope": False})
    if first1 and tape.vid(x) is None:
        raise RuntimeError("tape ffn: input must be a recorded value or declared input")
    vid1, hid = tape._out(0, (*x.shape[:-1], H), x.dtype, scale)
    seed1 = tape._seed() if drop_p > 0 else 0
    idx1 = tape._idx0(op1, hid.numel())
    if first1:
        op1.attrs["seed"] = seed1
        op1.attrs["K"] = C
    tape._finish(op1, [vid1], tape._req(op1, (mod1.weight, mod1.bias)))
    op2, first2 = tape._begin("linear", [hid, None], _linear_bw,
                              {"mod": mod2, "act": None, "p": float(drop_p), "relu_out": False, "rope": False})
    vid2, y = tape._out(0, (*x.shape[:-1], N), x.dtype, scale)
    seed2 = tape._seed() if drop_p > 0 else 0
    idx2 = tape._idx0(op2, y.numel())
    if first2:
        op2.attrs["seed"] = seed2
        op2.attrs["K"] = H
    tape._finish(op2, [vid2], tape._req(op2, (mod2.weight, mod2.bias)))
    ops.ffn_fwd(x.reshape(-1, C), w1, b1, w2, b2, drop_p, seed1, idx1, seed2, idx2, hid=hid.view(-1, H),
                y=y.view(-1, N))
    return y


def _linear_bw(tape, op, gys):
    (gy,) = gys
    mod, act, p = op.attrs["mod"], op.attrs["act"], op.attrs["p"]
    N, K = mod.compute_weight().shape
    gy2 = gy.view(-1, N)
    if op.attrs.get("rope") and op.outs[0] not in tape.derotated:  # rotate the output gradient back (in place)
        ropes = op.fattrs["rope"]
        c0 = tape.derotated_cols.get(op.outs[0], 0)  # columns the consumer already rotated back
        if c0:
            ropes = [r[:5] + (r[5] - c0, r[6]) for r in ropes]
        if all(r[2:] == ropes[0][2:] for r in ropes):
            ops.rope_blocks(gy2[:, c0:], ropes[0], inverse=True)
        else:
            st = tape.st(op.outs[0])
            for f, r in enumerate(ropes):
                ops.rope_blocks(gy[st.offsets[f]:st.offsets[f] + st.numels[f]].view(-1, N)[:, c0:], r, inverse=True)
    if op.outs[0] in tape.premasked:  # the consumer's dgrad already applied ReLU' and 1/keep
        dpre = gy2
    elif op.attrs["relu_out"]:
        dpre = ops.relu_mask_bwd(_flat(tape.st(op.outs[0]), N), gy2, 1.0 / (1.0 - p))
    elif p > 0:
        pre = tape.stores[("aux", op.idx, "pre")] if act else None
        dpre = ops.act_dropout_bwd(_flat(pre, N) if act else None, gy2, act, p, op.attrs["seed"])
    elif act:
        pre = tape.stores[("aux", op.idx, "pre")]
        dpre = ops.act_bwd(_flat(pre, N), gy2, act)
    else:
        dpre = gy2
    x2 = _flat(tape.st(op.ins[0]), K)
    wgrad = getattr(mod, "wgrad", None)
    gw, gb = mod.grad_views()
    with tape.side.run(dpre, x2):  # on the side stream: nothing below reads these gradients
        if wgrad is not None:  # a derived weight (functional.VFoldProj) scatters its own gradient
            wgrad(dpre, x2)
        elif gw is not None:
            ops.linear_wgrad(dpre, x2, gw.view(gw.shape[0], -1), db=gb)
        elif gb is not None:
            ops.colsum(dpre, gb)
    dx = None
    if op.needs[0] and op.idx in tape.prefused_dx:  # computed by the consumer's fused FFN backward
        dx = tape.prefused_dx.pop(op.idx)
    elif op.needs[0]:
        prod = tape.producer.get(op.ins[0])
        if prod is not None and prod.kind == "linear" and prod.attrs["relu_out"] and tape.nuse[op.ins[0]] == 1 \
                and op.ins[0] not in tape.seeded:
            # sole consumer of a ReLU (-> dropout) linear: its mask and 1/keep fused into this dgrad
            alpha = 1.0 / (1.0 - prod.attrs["p"])
            dx = _ffn_dgrad_fused(tape, op, prod, dpre, mod, x2, alpha)
            if dx is None:
                dx = _fp8.linear_dgrad(dpre, mod, pre=x2, act="relu", alpha=alpha).view(-1)
            tape.premasked.add(op.ins[0])
        elif not _ln_dgrad_fused(tape, op, prod, dpre, mod):
            dx = _dgrad_into(tape, op.ins[0], dpre, mod)
    dres = gy if op.needs[1] else None
    return [dx, dres]


def dgrad_acc_enabled():
    """S2H_DGRAD_ACC=0: a Linear's input gradient is always a new tensor, summed with the value's
    other gradients by a separate add (A/B of _dgrad_into)"""
    return os.environ.get("S2H_DGRAD_ACC", "1") != "0"


def _dgrad_into(tape, vid, dy, mod):
    """dx = dy @ W of a Linear whose input vid already holds a gradient from a later consumer: the
    dgrad GEMM's epilogue adds it (into it in place when this backward owns it, else as the residual
    of a new buffer) and the separate add launch goes; returns None then (nothing left to sum)"""
    prev = tape.grads.get(vid) if dgrad_acc_enabled() else None
    K = mod.compute_weight().shape[1]
    if (prev is None or prev.dtype != dy.dtype or dy.dtype != torch.bfloat16 or not prev.is_contiguous()
            or prev.numel() != dy.numel() // dy.shape[-1] * K or _fp8.dgrad_on_mx8(dy, mod)):
        return _fp8.linear_dgrad(dy, mod).view(-1)
    w = mod.compute_weight()
    if vid in tape.owned:
        ops.linear_dgrad(dy, w, dx=prev.view(-1, K), accumulate=True)
    else:
        tape.grads[vid] = ops.linear_dgrad(dy, w, residual=prev.view(-1, K)).view(-1)
        tape.owned.add(vid)
    return None


def ffn_fuse_enabled():
    """S2H_FFN_FUSE=0 runs the memory-attention FFN's input gradients as two GEMMs (dH with the ReLU /
    dropout mask in its epilogue, then dX = dH W1) instead of the one-launch ops.ffn_bwd_dgrad"""
    return os.environ.get("S2H_FFN_FUSE", "1") == "1"


def _ffn_dgrad_fused(tape, op, prod, dpre, mod, hid, alpha):
    """`op` = linear2 of a ReLU FFN whose linear1 is `prod` (memory_attention.py:97): compute both input
    gradients in one launch -- linear1's pre-activation gradient dH (returned, flat, as the gradient of
    hid; premasked) and linear1's input gradient dH W1 (handed to prod's backward through
    tape.prefused_dx).  None when the kernel does not apply (then the two-GEMM path runs)."""
    if not ffn_fuse_enabled() or not prod.needs[0]:
        return None
    mod1 = prod.attrs["mod"]
    if _fp8.dgrad_on_mx8(dpre, mod) or _fp8.dgrad_on_mx8(dpre, mod1):
        return None
    w2, w1 = mod.compute_weight(), mod1.compute_weight()
    if not ops.ffn_bwd_dgrad_ok(dpre, w2, w1, hid):
        return None
    dh, dx1 = ops.ffn_bwd_dgrad(dpre, w2, w1, hid, alpha)
    tape.prefused_dx[prod.idx] = dx1.view(-1)
    return dh.view(-1)


def ln_bwd_fuse_enabled():
    """S2H_LN_BWD_FUSE=1 fuses the LayerNorm backward into its consumer's dgrad (full-row tile).  Off
    by default for the same reason as functional.linear_ln_enabled: the full-row dgrad is slower than
    the 64-row-tile dgrad + the LayerNorm backward launch (bench step: 60.5 vs 59.6 ms per step,
    profiles/r04_v3_ln_fusion_ab.log)"""
    return os.environ.get("S2H_LN_BWD_FUSE", "0") == "1"


def _ln_dgrad_fused(tape, op, prod, dpre, mod):
    """The input of linear `op` is the output t of LayerNorm op `prod` and nothing else reads t
    (memory attention: norm1 -> q/k/v, norm2 -> cross-attention q, norm3 -> linear1): run the dgrad
    with the LayerNorm backward in its epilogue (ops.linear_dgrad_ln_bwd) -- dL/dt stays in registers
    -- and hand the LayerNorm's input gradients to its inputs here; `prod` is then left without
    output gradients (t has none, its residual-stream output's was consumed), so the backward walk
    skips it.  Needs the residual stream's gradient complete: every reader of it comes after `op`."""
    if prod is None or prod.kind != "ln" or not ln_bwd_fuse_enabled():
        return False
    t = op.ins[0]
    if prod.outs[0] != t or tape.nuse[t] != 1 or t in tape.seeded or _fp8.dgrad_on_mx8(dpre, mod):
        return False
    add = prod.attrs["add"]
    if add and tape.first_use.get(prod.outs[1], len(tape.ops)) <= op.idx:
        return False
    lnmod = prod.attrs["mod"]
    C = lnmod.weight.shape[0]
    w = mod.compute_weight()
    src = tape.st(prod.outs[1]) if add else tape.st(prod.ins[0])
    x2 = _flat(src, C)
    if w.shape[1] != C or not ops.linear_dgrad_ln_bwd_ok(dpre, w, x2):
        return False
    gxsum = tape.grads.pop(prod.outs[1], None) if add else None
    dx = ops.linear_dgrad_ln_bwd(dpre, w, x2, lnmod.weight.detach(), tape.stores[("aux", prod.idx, "mean")].buf,
                                 tape.stores[("aux", prod.idx, "rstd")].buf,
                                 dres=gxsum.contiguous().view(-1, C) if gxsum is not None else None,
                                 dgamma=_grad_of(lnmod.weight), dbeta=_grad_of(lnmod.bias)).view(-1)
    if prod.needs[0]:
        tape.acc(prod.ins[0], dx)
    if add and prod.needs[1]:
        tape.acc(prod.ins[1], dx)
    return True


def linear_add_ln(tape: FrameTape, inp, mod, x, norm, eps, drop_p):
    """(LN(x + y), x + y), y = drop(inp W^T + b), recorded as the two ops it replaces -- a linear
    (its output y a value that is never stored: the fused kernel keeps it in registers; its backward
    needs only the input and the dropout seed) and an add + LayerNorm (outputs LN(x + y), x + y; its
    backward reads x + y, mean, rstd) -- and run as ONE launch (ops.linear_add_ln)"""
    inp = inp if inp.is_contiguous() else inp.contiguous()
    x = x if x.is_contiguous() else x.contiguous()
    op, first = tape._begin("linear", [inp, None], _linear_bw,
                            {"mod": mod, "act": None, "p": float(drop_p), "relu_out": False, "rope": False})
    if first and tape.vid(inp) is None:
        raise RuntimeError("tape linear: input must be a recorded value or declared input")
    w = mod.compute_weight()
    N = w.shape[0]
    shape = (*inp.shape[:-1], N)
    vid, y = tape._out(0, shape, inp.dtype, tape._varlen_scale(inp))  # the never-written value y
    seed = tape._seed() if drop_p > 0 else 0
    idx0 = tape._idx0(op, y.numel())
    if first:
        op.attrs["seed"] = seed
        op.attrs["K"] = inp.shape[-1]
    tape._finish(op, [vid], tape._req(op, (mod.weight, mod.bias)))
    op2, _ = tape._begin("ln", [x, y], _ln_bw, {"mod": norm, "eps": eps, "add": True})
    rows = x.numel() // x.shape[-1]
    vt, t = tape._out(0, x.shape, x.dtype)
    vs, xsum = tape._out(1, x.shape, x.dtype)
    mean = tape._aux("mean", (rows,), torch.float32)
    rstd = tape._aux("rstd", (rows,), torch.float32)
    ops.linear_add_ln(inp, w, mod.compute_bias(), x, norm.weight.detach(), norm.bias.detach(), eps, drop_p=drop_p,
                      seed=seed, drop_idx0=idx0, xsum=xsum, y=t, mean=mean, rstd=rstd)
    tape._finish(op2, [vt, vs], tape._req(op2, (norm.weight, norm.bias)))
    return t, xsum


def mlp_heads(tape: FrameTape, pairs):
    """per-object MLP heads [(MLP, x)] as ONE op and one launch (ops.mlp_heads): outputs y per head;
    saved per head every hidden layer's ReLU output and, for a sigmoid head, the last pre-activation.
    The backward is the per-layer chain the separate linear ops would run (sigmoid' from the saved
    pre-activation, weight gradient, dgrad with the previous layer's ReLU' in its epilogue)"""
    xs = [x if x.is_contiguous() else x.contiguous() for _, x in pairs]
    mods = [m for m, _ in pairs]
    op, first = tape._begin("mlp_heads", xs, _mlp_heads_bw, {"mods": mods})
    if first and any(tape.vid(x) is None for x in xs):
        raise RuntimeError("tape mlp_heads: inputs must be recorded values or declared inputs")
    rows = xs[0].shape[0]
    vids, ys, hidden, pres, heads = [], [], [], [], []
    for hi, (m, x) in enumerate(zip(mods, xs)):
        layers = list(m.layers)
        vid, y = tape._out(hi, (rows, layers[-1].out_features), x.dtype)
        vids.append(vid)
        ys.append(y)
        hidden.append([tape._aux(f"h{hi}_{l}", (rows, layers[l].out_features), x.dtype) for l in range(len(layers) - 1)])
        pres.append(tape._aux(f"pre{hi}", (rows, layers[-1].out_features), x.dtype) if m.sigmoid_output else None)
        heads.append((x, [lin.compute_weight() for lin in layers], [lin.compute_bias() for lin in layers],
                      "sigmoid" if m.sigmoid_output else None))
    ops.mlp_heads(heads, outs=ys, hidden=hidden, pre=pres)
    params = [p for m in mods for lin in m.layers for p in (lin.weight, lin.bias)]
    tape._finish(op, vids, tape._req(op, params))
    return ys


def _mlp_heads_bw(tape, op, gys):
    dxs = []
    for hi, (m, gy) in enumerate(zip(op.attrs["mods"], gys)):
        if gy is None:
            dxs.append(None)
            continue
        layers = list(m.layers)
        L = len(layers)
        g = gy.view(-1, layers[-1].out_features)
        if m.sigmoid_output:
            g = ops.act_bwd(_flat(tape.stores[("aux", op.idx, f"pre{hi}")], layers[-1].out_features), g, "sigmoid")
        hs = [_flat(tape.stores[("aux", op.idx, f"h{hi}_{l}")], layers[l].out_features) for l in range(L - 1)]
        dx = None
        for l in range(L - 1, -1, -1):
            mod = layers[l]
            inp = _flat(tape.st(op.ins[hi]), layers[0].in_features) if l == 0 else hs[l - 1]
            gw, gb = mod.grad_views()
            if gw is not None:
                ops.linear_wgrad(g, inp, gw.view(gw.shape[0], -1), db=gb)
            elif gb is not None:
                ops.colsum(g, gb)
            if l > 0:  # the previous layer's ReLU' (from its output) in this dgrad's epilogue
                g = _fp8.linear_dgrad(g, mod, pre=hs[l - 1], act="relu", alpha=1.0)
            elif op.needs[hi]:
                dx = _fp8.linear_dgrad(g, mod).view(-1)
        dxs.append(dx)
    return dxs


# ---------------------------------------------------------------- layer norms
def layer_norm(tape: FrameTape, x, mod, eps, add=None, _compute=True):
    """LN(x) or (LN(x + add), x + add); _compute=False (no add): record only, returns (y, mean, rstd)"""
    x = x if x.is_contiguous() else x.contiguous()
    op, first = tape._begin("ln", [x, add], _ln_bw, {"mod": mod, "eps": eps, "add": add is not None})
    rows = x.numel() // x.shape[-1]
    vid, y = tape._out(0, x.shape, x.dtype)
    outs = [vid]
    xsum = None
    if add is not None:
        vid2, xsum = tape._out(1, x.shape, x.dtype)
        outs.append(vid2)
    mean = tape._aux("mean", (rows,), torch.float32)
    rstd = tape._aux("rstd", (rows,), torch.float32)
    if _compute:
        call_ln_fwd(x, mod, eps, y, mean, rstd, add, xsum)
    tape._finish(op, outs, tape._req(op, (mod.weight, mod.bias)))
    if not _compute:
        assert add is None
        return y, mean, rstd
    return (y, xsum) if add is not None else y


def layer_norm_pe_ok(x, mod, pe):
    """layer_norm_pe applies: bf16 rows of 256 (LayerNorm width), a contiguous bf16 [L, C] table
    whose L divides the rows, S2H_LN_PE not 0"""
    C = x.shape[-1]
    return (os.environ.get("S2H_LN_PE", "1") != "0" and x.dtype == torch.bfloat16 and pe.dtype == torch.bfloat16
            and C == 256 and x.is_contiguous() and mod.weight.shape[0] == C and pe.is_contiguous() and pe.dim() == 2 and pe.shape[1] == C
            and (x.numel() // C) % pe.shape[0] == 0)


def layer_norm_pe(tape: FrameTape, x, mod, eps, pe):
    """(LN(x), LN(x) + pe) in one launch (s2h_layernorm_fwd_pe): records the LayerNorm and the
    broadcast add of the constant table pe [L, C] (FN.add_bcast) as the two ops they replace"""
    y, mean, rstd = layer_norm(tape, x, mod, eps, _compute=False)
    k = add_bcast(tape, y, pe, 1.0, 1.0, None, None, _compute=False)
    C = x.shape[-1]
    from ._lib import call
    call("s2h_layernorm_fwd_pe", ops.dt(x), x.numel() // C, C, ops.ptr(x),
         ops.ptr(mod.weight.detach()), ops.ptr(mod.bias.detach()), float(eps), ops.ptr(y), ops.ptr(mean),
         ops.ptr(rstd), ops.ptr(pe), pe.shape[0], ops.ptr(k), ops.stream())
    return y, k


def call_ln_fwd(x, mod, eps, y, mean, rstd, add, xsum):
    from ._lib import call
    C = x.shape[-1]
    rows = x.numel() // C
    call("s2h_layernorm_fwd", ops.dt(x), rows, C, ops.ptr(x), C, ops.ptr(add), C, 0, ops.ptr(xsum),
         ops.ptr(mod.weight.detach()), ops.ptr(mod.bias.detach()), float(eps), ops.ptr(y), C, ops.ptr(mean),
         ops.ptr(rstd), ops.stream())


def _ln_bw(tape, op, gys):
    gy = gys[0]
    gxsum = gys[1] if len(gys) > 1 else None
    mod = op.attrs["mod"]
    k = op.idx
    C = mod.weight.shape[0]
    src = tape.st(op.outs[1]) if op.attrs["add"] else tape.st(op.ins[0])
    x2 = _flat(src, C)
    mean = tape.stores[("aux", k, "mean")].buf
    rstd = tape.stores[("aux", k, "rstd")].buf
    if gy is None:
        gy = torch.zeros_like(src.buf)
    dx = ops.layernorm_bwd(x2, gy.view(-1, C), mod.weight.detach(), mean, rstd,
                           dres=gxsum.contiguous().view(-1, C) if gxsum is not None else None,
                           dgamma=_grad_of(mod.weight), dbeta=_grad_of(mod.bias))
    dx = dx.view(-1)
    return [dx, dx if op.attrs["add"] else None]


# ---------------------------------------------------------------- attention
def attention(tape: FrameTape, q, k, v, scale, p_drop, _compute=True):
    """q [B, Lq, H, D], k / v [B, Lk, H, D] views of recorded values (contiguous per value);
    _compute=False: record only, returns (o, lse)"""
    op, first = tape._begin("attn", [q, k, v], _attn_bw, {"scale": scale, "p": p_drop})
    B, Lq, H, D = q.shape
    Lk = k.shape[1]
    vid, o = tape._out(0, (B, Lq, H, D), q.dtype)
    lse = tape._aux("lse", (B, H, Lq), torch.float32)
    seed = tape._seed() if p_drop > 0 else 0
    idx0 = tape._idx0(op, B * H * Lq * Lk)
    keep = tape._keep_bits(q, Lk, op.ins[1], p_drop)
    if _compute:
        ops.attn_fwd(q, k, v, o, lse, scale, p_drop, seed, idx0=idx0, keep=keep)
    else:
        assert p_drop == 0 and keep is None
    tape._fattr(op, "Lk", Lk)
    if first:
        op.attrs.update(seed=seed, B=B, Lq=Lq, H=H, D=D, qshape=tuple(q.shape), keep=keep is not None)
    tape._finish(op, [vid], any(op.needs))
    return o if _compute else (o, lse)


def _attn_frames_bwd(tape, op, q_all, k_st, v_st, kview, o_all, go, lse, dq, dk_buf, dv_buf, rope=None):
    """one frame-table flash launch, or a per-frame loop of the generic kernels; rope (flash launch
    only, see ops.flash_bwd_frames): True when the launch rotated dq / dk back"""
    a = op.attrs
    F, B, Lq, H, D = tape.F, a["B"], a["Lq"], a["H"], a["D"]
    lks = op.fattrs["Lk"]
    krow = [0]
    for f in range(F - 1):
        krow.append(krow[-1] + B * lks[f])
    k_rows, v_rows, dk_rows, dv_rows = kview
    ks = tape.stores[("aux", op.idx, "keep")] if a.get("keep") else None
    if ops.flash_bwd_eligible(q_all):
        ops.flash_bwd_frames(F, B, lks, krow, op.fattrs["idx0"], q_all, k_rows, v_rows, o_all, go, lse, dq,
                             dk_rows, dv_rows, a["scale"], a["p"], a["seed"], keep=ks.buf if ks else None,
                             koff=ks.offsets if ks else None, rope=rope)
        return rope is not None
    assert ks is None, "keep bitmap written but the flash backward is not eligible"
    if len(set(lks)) == 1:
        # uniform key count: the frames ARE one [F*B] batch (frame f's dropout indices start at
        # f*B*H*Lq*Lk, where its forward put them)
        Lk = lks[0]
        ops.attn_bwd(q_all, k_rows.view(F * B, Lk, H, D), v_rows.view(F * B, Lk, H, D), o_all, go, lse, dq,
                     dk_rows.view(F * B, Lk, H, D), dv_rows.view(F * B, Lk, H, D), a["scale"], a["p"], a["seed"])
        return
    for f in range(F):
        sl = slice(f * B, (f + 1) * B)
        r0, r1 = krow[f], krow[f] + B * lks[f]
        ops.attn_bwd(q_all[sl], k_rows[r0:r1].view(B, lks[f], H, D), v_rows[r0:r1].view(B, lks[f], H, D), o_all[sl],
                     go[sl], lse[sl], dq[sl], dk_rows[r0:r1].view(B, lks[f], H, D),
                     dv_rows[r0:r1].view(B, lks[f], H, D), a["scale"], a["p"], a["seed"], idx0=op.fattrs["idx0"][f])


def _attn_bw(tape, op, gys):
    (go,) = gys
    a = op.attrs
    F, B, Lq, H, D = tape.F, a["B"], a["Lq"], a["H"], a["D"]
    k_idx = op.idx
    q_st, k_st, v_st = (tape.st(v) for v in op.ins)
    q_all = q_st.buf.view(F * B, Lq, H, D)
    o_all = tape.st(op.outs[0]).buf.view(F * B, Lq, H, D)
    go = go.contiguous().view(F * B, Lq, H, D)
    lse = tape.stores[("aux", k_idx, "lse")].buf.view(F * B, H, Lq)
    dq = torch.empty_like(q_all)
    dk = torch.empty(k_st.buf.numel(), device=go.device, dtype=go.dtype)
    dv = torch.empty(v_st.buf.numel(), device=go.device, dtype=go.dtype)
    rows = lambda t: t.view(-1, H, D)  # noqa: E731
    _attn_frames_bwd(tape, op, q_all, k_st, v_st, (rows(k_st.buf), rows(v_st.buf), rows(dk), rows(dv)), o_all, go,
                     lse, dq, dk, dv)
    return [dq.view(-1), dk, dv]


def attention_vfold(tape: FrameTape, q, k, mem, scale, p_drop):
    """the folded cross-attention (functional.attention_vfold): q [B, Lq, 1, 256], k [B, Lk, 1, 256],
    mem [B, Lk, 1, 64] views of recorded values -> u' [B, Lq, 1, 72]"""
    op, first = tape._begin("attn_vfold", [q, k, mem], _attn_vfold_bw, {"scale": scale, "p": p_drop})
    B, Lq = q.shape[0], q.shape[1]
    Lk = k.shape[1]
    vid, u = tape._out(0, (B, Lq, 1, ops.VFOLD_COLS), q.dtype)
    lse = tape._aux("lse", (B, 1, Lq), torch.float32)
    seed = tape._seed() if p_drop > 0 else 0
    idx0 = tape._idx0(op, B * Lq * Lk)
    keep = tape._keep_bits(q, Lk, op.ins[1], p_drop)
    ops.attn_fwd_vfold(q, k, mem, u, lse, scale, p_drop, seed, idx0=idx0, keep=keep)
    tape._fattr(op, "Lk", Lk)
    if first:
        op.attrs.update(seed=seed, B=B, Lq=Lq, D=q.shape[-1], keep=keep is not None)
    tape._finish(op, [vid], any(op.needs))
    return u


def _attn_vfold_bw(tape, op, gys):
    (gu,) = gys
    a = op.attrs
    F, B, Lq, D = tape.F, a["B"], a["Lq"], a["D"]
    q_st, k_st, m_st = (tape.st(v) for v in op.ins)
    q_all = q_st.buf.view(F * B, Lq, 1, D)
    u_all = tape.st(op.outs[0]).buf.view(F * B, Lq, 1, ops.VFOLD_COLS)
    gu = gu.contiguous().view(F * B, Lq, 1, ops.VFOLD_COLS)
    lse = tape.stores[("aux", op.idx, "lse")].buf.view(F * B, 1, Lq)
    dq = torch.empty_like(q_all)
    dk = torch.empty(k_st.buf.numel(), device=gu.device, dtype=gu.dtype)
    lks = op.fattrs["Lk"]
    krow = [0]
    for f in range(F - 1):
        krow.append(krow[-1] + B * lks[f])
    ks = tape.stores[("aux", op.idx, "keep")] if a.get("keep") else None
    rope = _vfold_k_rope(tape, op.ins[1], lks, D)
    # the q projection's RoPE (transformer.py:296) into the dQ store when it uses the same tables
    rq = _proj_rope(tape, op.ins[0], [Lq] * F, D, D) if bwd_rope_fuse_enabled() else None
    if rq is not None and rope is not None and (rq[0] is not rope[0] or rq[1] is not rope[1] or rq[2] != rope[2]):
        rq = None
    if rope is None and rq is not None:
        rope = (rq[0], rq[1], rq[2], None)
    ops.flash_bwd_frames_vfold(F, B, lks, krow, op.fattrs["idx0"], q_all, k_st.buf.view(-1, 1, D),
                               m_st.buf.view(-1, 1, ops.VFOLD_DV), u_all, gu, lse, dq, dk.view(-1, 1, D), a["scale"],
                               a["p"], a["seed"], keep=ks.buf if ks else None, koff=ks.offsets if ks else None,
                               rope=rope, rope_q=rq[3] if rq else None)
    if rope is not None and rope[3] is not None:
        tape.derotated.add(op.ins[1])
    if rq is not None:
        tape.derotated.add(op.ins[0])
    return [dq.view(-1), dk, None]


def _vfold_k_rope(tape, kvid, lks, D):
    """(cos, sin, period, nrot per frame) when the keys are the output of ONE linear-with-RoPE op
    (the cross-attention's k projection, RoPE in its epilogue), used by this attention only, one
    head of D columns rotated in full, one L-row block per object -- the dK store then rotates the
    gradient back and the linear's backward skips its rope pass; else None"""
    if os.environ.get("S2H_VFOLD_DK_ROPE", "1") == "0":
        return None
    return _proj_rope(tape, kvid, lks, D, D)


def bwd_rope_fuse_enabled():
    """S2H_BWD_ROPE_FUSE=0 keeps the q (and self-attention k) projections' inverse RoPE as separate
    passes in the linear backward instead of the attention backward's dQ / dK stores"""
    return os.environ.get("S2H_BWD_ROPE_FUSE", "1") != "0"


def _proj_rope(tape, vid, rows, D, ncol):
    """(cos, sin, period, rotated rows per frame) when value vid is the output of ONE linear-with-RoPE
    op used by one attention only, whose epilogue rotates D-wide heads over its first ncol columns in
    blocks of rows[f] rows with the same tables in every frame; else None"""
    prod = tape.producer.get(vid)
    if prod is None or prod.kind != "linear" or tape.nuse[vid] != 1:
        return None
    ropes = prod.fattrs.get("rope")
    if not ropes or len(ropes) != len(rows) or any(r is None for r in ropes):
        return None
    cos, sin, _, _, period, _, _ = ropes[0]
    for f, r in enumerate(ropes):
        if r[0] is not cos or r[1] is not sin or r[4] != period or r[5] != ncol or r[6] != D or r[2] != rows[f]:
            return None
    return cos, sin, period, [r[3] for r in ropes]


def qkv_attention(tape: FrameTape, qkv, scale, p_drop, rope):
    """self-attention on a packed [B, L, 3, H, d] projection (optional RoPE on q and k)"""
    op, first = tape._begin("qkv_attn", [qkv], _qkv_bw, {"scale": scale, "p": p_drop, "rope": rope})
    B, L, _, H, D = qkv.shape
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    if rope is not None:
        cos, sin, period = rope
        qk = tape._aux("qk", (B, L, 2, H, D), qkv.dtype)
        _rope_into(q, qk[:, :, 0], L, cos, sin, period)
        _rope_into(k, qk[:, :, 1], L, cos, sin, period)
        q, k = qk[:, :, 0], qk[:, :, 1]
    vid, o = tape._out(0, (B, L, H, D), qkv.dtype)
    lse = tape._aux("lse", (B, H, L), torch.float32)
    seed = tape._seed() if p_drop > 0 else 0
    idx0 = tape._idx0(op, B * H * L * L)
    keep = tape._keep_bits(q, L, None, p_drop)
    ops.attn_fwd(q, k, v, o, lse, scale, p_drop, seed, idx0=idx0, keep=keep)
    tape._fattr(op, "Lk", L)
    if first:
        op.attrs.update(seed=seed, B=B, Lq=L, H=H, D=D, keep=keep is not None)
    tape._finish(op, [vid], any(op.needs))
    return o


def _rope_into(x, y, nrot, cos, sin, period, inverse=False):
    """rotate rows < nrot of x [B, L, H, D] (strided) into y [B, L, H, D] (strided)"""
    from ._lib import call
    B, L, H, D = x.shape
    assert H == 1 or (x.stride(2) == D and y.stride(2) == D)
    call("s2h_rope", ops.dt(x), B, int(nrot), H * D, ops.ptr(x), x.stride(0), x.stride(1), ops.ptr(y), y.stride(0),
         y.stride(1), ops.ptr(cos), ops.ptr(sin), int(period), int(inverse), ops.stream())


def _qkv_bw(tape, op, gys):
    (go,) = gys
    a = op.attrs
    F, B, L, H, D = tape.F, a["B"], a["Lq"], a["H"], a["D"]
    k_idx = op.idx
    qkv_all = tape.st(op.ins[0]).buf.view(F * B, L, 3, H, D)
    rope = a["rope"]
    if rope is not None:
        qk_all = tape.stores[("aux", k_idx, "qk")].buf.view(F * B, L, 2, H, D)
        q_all, k_all = qk_all[:, :, 0], qk_all[:, :, 1]
    else:
        q_all, k_all = qkv_all[:, :, 0], qkv_all[:, :, 1]
    v_all = qkv_all[:, :, 2]
    o_all = tape.st(op.outs[0]).buf.view(F * B, L, H, D)
    lse = tape.stores[("aux", k_idx, "lse")].buf.view(F * B, H, L)
    dqkv = torch.empty(qkv_all.shape, device=go.device, dtype=go.dtype)
    dq, dk, dv = dqkv[:, :, 0], dqkv[:, :, 1], dqkv[:, :, 2]
    go = go.contiguous().view(F * B, L, H, D)
    def rows(t):  # [F*B, L, H, D] slice of a packed projection -> [F*B*L, H, D] rows (uniform row stride)
        assert t.stride(0) == L * t.stride(1)
        return torch.as_strided(t, (F * B * L, H, D), (t.stride(1), t.stride(2), 1), t.storage_offset())
    # the qkv projection's RoPE epilogue on q (its first D columns) transposed into the dQ store when
    # this attention is its only consumer; the linear's backward then rotates only the k columns
    fuse = None
    if rope is None and H == 1 and D == 256 and bwd_rope_fuse_enabled():
        pr = _proj_rope(tape, op.ins[0], [L] * F, D, 2 * D)
        if pr is not None:
            fuse = (pr[0], pr[1], pr[2], pr[3])
    if _attn_frames_bwd(tape, op, q_all, None, None, (rows(k_all), rows(v_all), rows(dk), rows(dv)), o_all, go, lse,
                        dq, None, None, rope=fuse):
        tape.derotated_cols[op.ins[0]] = D
    if rope is not None:
        cos, sin, period = rope
        for g in (dq, dk):
            _rope_into(g, g, L, cos, sin, period, inverse=True)
    return [dqkv.view(-1)]


# ---------------------------------------------------------------- RoPE
def rope(tape: FrameTape, x, nrot, cos, sin, period):
    """x [Bt, L, D]: rotate rows < nrot (per frame: the memory rows of the frame), copy the rest"""
    x = x if x.is_contiguous() else x.contiguous()
    op, first = tape._begin("rope", [x], _rope_bw, {"cos": cos, "sin": sin, "period": period})
    scale = tape._varlen_scale(x)
    vid, y = tape._out(0, x.shape, x.dtype, scale)
    if nrot < x.shape[1]:
        y[:, nrot:].copy_(x[:, nrot:])
    ops.rope(x, y, nrot, cos, sin, period)
    tape._fattr(op, "nrot", int(nrot))
    tape._fattr(op, "shape", tuple(x.shape))
    tape._finish(op, [vid], any(op.needs))
    return y


def _rope_bw(tape, op, gys):
    (gy,) = gys
    a = op.attrs
    out_st = tape.st(op.outs[0])
    dx = torch.empty_like(gy)
    shapes, nrots = op.fattrs["shape"], op.fattrs["nrot"]
    if out_st.uniform and len(set(nrots)) == 1:
        Bt, L, D = shapes[0]
        g3 = gy.view(-1, L, D)
        d3 = dx.view(-1, L, D)
        if nrots[0] < L:
            d3[:, nrots[0]:].copy_(g3[:, nrots[0]:])
        ops.rope(g3, d3, nrots[0], a["cos"], a["sin"], a["period"], inverse=True)
        return [dx]
    for f in range(tape.F):
        o, n = out_st.offsets[f], out_st.numels[f]
        g3 = gy[o:o + n].view(shapes[f])
        d3 = dx[o:o + n].view(shapes[f])
        nr = nrots[f]
        if nr < shapes[f][1]:
            d3[:, nr:].copy_(g3[:, nr:])
        ops.rope(g3, d3, nr, a["cos"], a["sin"], a["period"], inverse=True)
    return [dx]


# ---------------------------------------------------------------- elementwise
def add(tape: FrameTape, a, b, alpha, beta, _compute=True):
    a = a if a.is_contiguous() else a.contiguous()
    b = b if b.is_contiguous() else b.contiguous()
    op, first = tape._begin("add", [a, b], _add_bw, {"alpha": alpha, "beta": beta})
    scale = tape._varlen_scale(a, b)
    vid, out = tape._out(0, a.shape, a.dtype, scale)
    if _compute:
        ops.add(a, b, out=out, alpha=alpha, beta=beta)
    tape._finish(op, [vid], any(op.needs))
    return out


def _scaled(g, s):
    return g if s == 1.0 else ops.add(g, None, alpha=s)


def _add_bw(tape, op, gys):
    (g,) = gys
    return [_scaled(g, op.attrs["alpha"]) if op.needs[0] else None,
            _scaled(g, op.attrs["beta"]) if op.needs[1] else None]


def add_bcast(tape: FrameTape, a, b, alpha, beta, shape, bparam, _compute=True):
    """out[o, ...] = alpha a[o, ...] + beta b[...]; b is a constant table, a parameter's compute
    copy (bparam) or a recorded value (the memory positional table); _compute=False: record only"""
    a = a if (a is None or a.is_contiguous()) else a.contiguous()
    b = b.contiguous()
    op, first = tape._begin("add_bcast", [a, b], _add_bcast_bw, {"alpha": alpha, "beta": beta, "bparam": bparam})
    scale = tape._varlen_scale(a, b)
    oshape = a.shape if a is not None else shape
    vid, out = tape._out(0, oshape, b.dtype, scale)
    if _compute:
        ops.add_bcast(a, b, out=out, alpha=alpha, beta=beta)
    tape._fattr(op, "inner", b.numel())
    tape._fattr(op, "outer", out.numel() // b.numel())
    tape._finish(op, [vid], tape._req(op, (bparam,)))
    return out


def _add_bcast_bw(tape, op, gys):
    (g,) = gys
    a = op.attrs
    da = _scaled(g, a["alpha"]) if op.needs[0] else None
    db = None
    inners, outers = op.fattrs["inner"], op.fattrs["outer"]
    if a["bparam"] is not None:
        gb = _grad_of(a["bparam"])
        if gb is not None:
            inner = inners[0]
            tmp = None
            if a["beta"] != 1.0:
                tmp = torch.zeros(inner, device=g.device, dtype=torch.float32)
                ops.colsum(g.view(-1, inner), tmp)
                ops.add(gb.view(-1), tmp, beta=a["beta"], out=gb.view(-1))
            else:
                ops.colsum(g.view(-1, inner), gb.view(-1), accumulate=True)
    elif op.needs[1]:
        bst = tape.st(op.ins[1])
        db = torch.empty(bst.buf.numel(), device=g.device, dtype=g.dtype)
        go = 0
        for f in range(tape.F):
            n_in, n_out = inners[f], inners[f] * outers[f]
            ops.sum_outer(g[go:go + n_out].view(outers[f], n_in), db[bst.offsets[f]:bst.offsets[f] + n_in])
            go += n_out
        if a["beta"] != 1.0:
            db = ops.add(db, None, alpha=a["beta"])
    return [da, db]


def act(tape: FrameTape, x, a, _compute=True):
    x = x if x.is_contiguous() else x.contiguous()
    op, first = tape._begin("act", [x], _act_bw, {"act": a})
    vid, out = tape._out(0, x.shape, x.dtype)
    if _compute:
        ops.act_fwd(x, a, out=out)
    tape._finish(op, [vid], any(op.needs))
    return out


def _act_bw(tape, op, gys):
    (g,) = gys
    return [ops.act_bwd(tape.st(op.ins[0]).buf, g.contiguous().view(-1), op.attrs["act"])]


def cast(tape: FrameTape, x, dtype):
    x = x if x.is_contiguous() else x.contiguous()
    op, first = tape._begin("cast", [x], _cast_bw, {"src": x.dtype})
    vid, out = tape._out(0, x.shape, dtype)
    ops.cast(x, dtype, out=out)
    tape._finish(op, [vid], any(op.needs))
    return out


def _cast_bw(tape, op, gys):
    (g,) = gys
    return [ops.cast(g.contiguous().view(-1), op.attrs["src"])]


def expand_batch(tape: FrameTape, x, O):
    """[1, ...] -> [O, ...] materialised broadcast (grad = sum over O)"""
    x = x if x.is_contiguous() else x.contiguous()
    op, first = tape._begin("expand", [x], _expand_bw, {"O": O})
    vid, out = tape._out(0, (O, *x.shape[1:]), x.dtype)
    ops.add_bcast(None, x, out=out)
    tape._finish(op, [vid], any(op.needs))
    return out


def _expand_bw(tape, op, gys):
    (g,) = gys
    O = op.attrs["O"]
    inner = tape.st(op.ins[0]).numels[0]
    d = torch.empty(tape.F * inner, device=g.device, dtype=g.dtype)
    ops.sum_outer_batched(g.contiguous().view(tape.F, O, inner), d)  # every frame in one launch
    return [d]


def row_gate(tape: FrameTape, x, gate, fill):
    """x[r] if gate[r] > 0 else fill; gate [R] f32 per-frame constant (no gradient)"""
    x = x if x.is_contiguous() else x.contiguous()
    op, first = tape._begin("row_gate", [x], _row_gate_bw, {"fill": fill})
    vid, out = tape._out(0, x.shape, x.dtype)
    gsave = tape._aux("gate", gate.shape, gate.dtype)
    gsave.copy_(gate)
    ops.row_gate(x, gate, fill, out=out)
    tape._finish(op, [vid], any(op.needs))
    return out


def cast_gate(tape: FrameTape, x, dtype, gate, fill):
    """row_gate(cast(x, dtype), gate, fill) as one op and one launch (s2h_row_gate_cast, which also
    saves the gate); backward: gate > 0 ? g : 0 cast back to x's dtype in one launch"""
    x = x if x.is_contiguous() else x.contiguous()
    op, first = tape._begin("cast_gate", [x], _cast_gate_bw, {"src": x.dtype})
    vid, out = tape._out(0, x.shape, dtype)
    gsave = tape._aux("gate", gate.shape, gate.dtype)
    ops.row_gate_cast(x, gate, fill, dtype, out=out, gate_out=gsave)
    tape._finish(op, [vid], any(op.needs))
    return out


def _cast_gate_bw(tape, op, gys):
    (g,) = gys
    gate = tape.stores[("aux", op.idx, "gate")].buf
    R = gate.numel()
    return [ops.row_gate_cast(g.contiguous().view(R, -1), gate, 0.0, op.attrs["src"], backward=True).view(-1)]


def _row_gate_bw(tape, op, gys):
    (g,) = gys
    gate = tape.stores[("aux", op.idx, "gate")].buf
    R = gate.numel()
    return [ops.row_gate(g.contiguous().view(R, -1), gate, 0.0, backward=True).view(-1)]


def bilinear(tape: FrameTape, x, ho, wo):
    x = x if x.is_contiguous() else x.contiguous()
    op, first = tape._begin("bilinear", [x], _bilinear_bw, {"hw": tuple(x.shape[-2:])})
    vid, out = tape._out(0, (*x.shape[:-2], ho, wo), x.dtype)
    ops.bilinear(x, ho, wo, out=out)
    tape._finish(op, [vid], any(op.needs))
    return out


def _bilinear_bw(tape, op, gys):
    (g,) = gys
    hi, wi = op.attrs["hw"]
    out_shape = tape.st(op.outs[0]).shape0
    g3 = g.contiguous().view(-1, out_shape[-2], out_shape[-1])
    return [ops.bilinear_bwd(g3, hi, wi).view(-1)]


def select_token(tape: FrameTape, x, i):
    """x [B, N, C] -> x[:, i] (contiguous copy)"""
    op, first = tape._begin("select", [x], _select_bw, {"i": i, "shape": tuple(x.shape)})
    B, N, C = x.shape
    vid, out = tape._out(0, (B, C), x.dtype)
    out.copy_(x[:, i])
    tape._finish(op, [vid], any(op.needs))
    return out


def select_tokens_ok(x):
    """select_tokens applies: 16-B aligned token rows (ops.copy_segments' batched 2-D copies)"""
    return (os.environ.get("S2H_SELECT_N", "1") != "0" and x.dim() == 3 and x.is_contiguous()
            and (x.shape[-1] * x.element_size()) % 16 == 0 and x.data_ptr() % 16 == 0)


def select_tokens(tape: FrameTape, x, idxs):
    """x [B, N, C] -> [x[:, i] for i in idxs] (contiguous copies) as one op: one batched copy launch
    forward (ops.copy_segments), one zero fill + one batched copy backward"""
    op, first = tape._begin("select_n", [x], _select_n_bw, {"idxs": tuple(idxs), "shape": tuple(x.shape)})
    B, N, C = x.shape
    vids, outs = [], []
    for j in range(len(idxs)):
        vid, out = tape._out(j, (B, C), x.dtype)
        vids.append(vid)
        outs.append(out)
    ops.copy_segments([(x[:, i], out) for i, out in zip(idxs, outs)])
    tape._finish(op, vids, any(op.needs))
    return outs


def _select_n_bw(tape, op, gys):
    B, N, C = op.attrs["shape"]
    ref = next(g for g in gys if g is not None)
    d = torch.zeros(tape.F * B, N, C, device=ref.device, dtype=ref.dtype)
    ops.copy_segments([(g.contiguous().view(tape.F * B, C), d[:, i]) for i, g in zip(op.attrs["idxs"], gys)
                       if g is not None])
    return [d.view(-1)]


def _select_bw(tape, op, gys):
    (g,) = gys
    B, N, C = op.attrs["shape"]
    d = torch.zeros(tape.F * B, N, C, device=g.device, dtype=g.dtype)
    d[:, op.attrs["i"]].copy_(g.view(tape.F * B, C))
    return [d.view(-1)]


# ---------------------------------------------------------------- SAM pieces
def conv_transpose2x2(tape: FrameTape, x, mod, add=None, _compute=True):
    """ConvTranspose2d(2, 2) + bias (+ add broadcast over the batch when it has batch 1);
    _compute=False: record only, returns the output slot"""
    x = x if x.is_contiguous() else x.contiguous()
    op, first = tape._begin("convt", [x, add], _convt_bw, {"mod": mod})
    B, H, W, Ci = x.shape
    Co = mod.out_ch
    if not _compute:
        vid, out = tape._out(0, (B, 2 * H, 2 * W, Co), x.dtype)
        if first:
            op.attrs.update(B=B, H=H, W=W, Ci=Ci, Co=Co, bcast=add is not None and add.shape[0] != B)
        tape._finish(op, [vid], tape._req(op, (mod.weight, mod.bias)))
        return out
    w = mod.compute_weight()
    # the GEMM output is scratch: the backward needs only x and the output gradient
    Y = torch.empty(B * H * W, 4 * Co, device=x.device, dtype=x.dtype)
    ops.gemm(x.reshape(-1, Ci), w, Y, M=B * H * W, N=4 * Co, K=Ci, lda_m=Ci, lda_k=1, ldb_k=4 * Co, ldb_n=1,
             ldc=4 * Co)
    vid, out = tape._out(0, (B, 2 * H, 2 * W, Co), x.dtype)
    if ops.convt2_direct() and Co % (16 // x.element_size()) == 0:  # scatter + bias + add, one launch
        ops.convt2_store(Y, B, H, W, Co, bias=mod.bias.detach(), add=None if add is None else add.contiguous(),
                         out=out)
    else:
        ops.convt2_scatter(Y, B, H, W, Co, bias=mod.bias.detach(), add=None, out=out)
        if add is not None:
            add = add.contiguous()
            if add.shape[0] == B:
                ops.add(out, add, out=out)
            else:
                ops.add_bcast(out, add, out=out)
    if first:
        op.attrs.update(B=B, H=H, W=W, Ci=Ci, Co=Co, bcast=add is not None and add.shape[0] != B)
    tape._finish(op, [vid], tape._req(op, (mod.weight, mod.bias)))
    return out


def _convt_bw(tape, op, gys):
    (g,) = gys
    a = op.attrs
    mod, F = a["mod"], tape.F
    B, H, W, Ci, Co = a["B"], a["H"], a["W"], a["Ci"], a["Co"]
    g = g.contiguous()
    dY = ops.convt2_gather(g.view(F * B, 2 * H, 2 * W, Co), F * B, H, W, Co)
    gw, gb = _grad_of(mod.weight), _grad_of(mod.bias)
    x2 = _flat(tape.st(op.ins[0]), Ci)
    R = F * B * H * W
    if gw is not None:
        ops.gemm(x2, dY, gw.view(Ci, 4 * Co), M=Ci, N=4 * Co, K=R, lda_m=1, lda_k=Ci, ldb_k=4 * Co, ldb_n=1,
                 ldc=4 * Co, beta=1.0)
    if gb is not None:
        ops.colsum(g.view(-1, Co), gb)
    dx = None
    if op.needs[0]:
        dx = torch.empty(R * Ci, device=g.device, dtype=g.dtype)
        ops.gemm(dY, mod.compute_weight(), dx.view(R, Ci), M=R, N=Ci, K=4 * Co, lda_m=4 * Co, lda_k=1, ldb_k=1,
                 ldb_n=4 * Co, ldc=Ci)
    dadd = None
    if op.needs[1]:
        if a["bcast"]:
            inner = 4 * H * W * Co
            dadd = torch.empty(F * inner, device=g.device, dtype=g.dtype)
            ops.sum_outer_batched(g.view(F, B, inner), dadd)  # every frame in one launch
        else:
            dadd = g.view(-1)
    return [dx, dadd]


def hyper_mask(tape: FrameTape, hyper, up, _compute=True):
    """masks[o, p] = sum_c hyper[o, c] up[o, p, c]"""
    hyper = hyper if hyper.is_contiguous() else hyper.contiguous()
    op, first = tape._begin("hyper", [hyper, up], _hyper_bw, {})
    O, P, C = up.shape
    vid, out = tape._out(0, (O, P), up.dtype)
    if _compute:
        ops.bmm(hyper.view(O, 1, C), up, out.view(O, 1, P), trans_b=True)
    if first:
        op.attrs.update(O=O, P=P, C=C)
    tape._finish(op, [vid], any(op.needs))
    return out


def _hyper_bw(tape, op, gys):
    (g,) = gys
    F, O, P, C = tape.F, op.attrs["O"], op.attrs["P"], op.attrs["C"]
    h3 = tape.st(op.ins[0]).buf.view(F * O, 1, C)
    up = tape.st(op.ins[1]).buf.view(F * O, P, C)
    g3 = g.contiguous().view(F * O, 1, P)
    dh = dup = None
    if op.needs[0]:
        dh32 = torch.empty(F * O, 1, C, device=g.device, dtype=torch.float32)
        ops.bmm(g3, up, dh32)
        dh = ops.cast(dh32, up.dtype).view(-1)
    if op.needs[1]:
        dup = torch.empty(F * O, P, C, device=g.device, dtype=up.dtype)
        ops.gemm(g3, h3, dup, M=P, N=C, K=1, lda_m=1, lda_k=P, ldb_k=C, ldb_n=1, ldc=C, batch=F * O, sA=P, sB=C,
                 sC=P * C)
        dup = dup.view(-1)
    return [dh, dup]


def convt_tail_ok(x, mod, add, hyper):
    return (ops.convt2_tail_enabled() and x.dtype == torch.bfloat16 and mod.out_ch == 32 and hyper.dim() == 2
            and hyper.shape == (x.shape[0], 32) and (add is None or add.shape[1:] == (2 * x.shape[1], 2 * x.shape[2], 32)))


def convt_tail(tape: FrameTape, x, mod, add, hyper):
    """masks = hyper_mask(hyper, gelu(conv_transpose2x2(x, mod, add))) (mask_decoder.py:105-113) as
    one GEMM + one launch (s2h_convt2_tail), recorded as the same three tape ops (convt, act, hyper)
    with their saved values, so the frame-batched backward is unchanged"""
    x = x if x.is_contiguous() else x.contiguous()
    hyper = hyper if hyper.is_contiguous() else hyper.contiguous()
    add = None if add is None else add.contiguous()
    B, H, W, Ci = x.shape
    Co = mod.out_ch
    pre = conv_transpose2x2(tape, x, mod, add=add, _compute=False)
    post = act(tape, pre, "gelu", _compute=False)
    masks = hyper_mask(tape, hyper, post.view(B, -1, Co), _compute=False)
    Y = torch.empty(B * H * W, 4 * Co, device=x.device, dtype=x.dtype)  # scratch
    ops.gemm(x.reshape(-1, Ci), mod.compute_weight(), Y, M=B * H * W, N=4 * Co, K=Ci, lda_m=Ci, lda_k=1,
             ldb_k=4 * Co, ldb_n=1, ldc=4 * Co)
    ops.convt2_tail(Y, B, H, W, Co, mod.bias.detach(), add, hyper, pre, post, masks)
    return masks


def convt_ln_gelu_ok(x, mod, add, ln):
    return (ops.convt2_tail_enabled() and x.dtype == torch.bfloat16 and mod.out_ch == 64
            and ln.weight.shape[0] == 64 and (add is None or add.shape[1:] == (2 * x.shape[1], 2 * x.shape[2], 64)))


def convt_ln_gelu(tape: FrameTape, x, mod, add, ln):
    """gelu(ln(conv_transpose2x2(x, mod, add))) (mask_decoder.py:105-106) as one GEMM + one launch
    (s2h_convt2_ln_gelu), recorded as the same three tape ops (convt, ln, act) with their saved values"""
    x = x if x.is_contiguous() else x.contiguous()
    add = None if add is None else add.contiguous()
    B, H, W, Ci = x.shape
    Co = mod.out_ch
    pre = conv_transpose2x2(tape, x, mod, add=add, _compute=False)
    y, mean, rstd = layer_norm(tape, pre, ln, ln.eps, _compute=False)
    post = act(tape, y, "gelu", _compute=False)
    Y = torch.empty(B * H * W, 4 * Co, device=x.device, dtype=x.dtype)  # scratch
    ops.gemm(x.reshape(-1, Ci), mod.compute_weight(), Y, M=B * H * W, N=4 * Co, K=Ci, lda_m=Ci, lda_k=1,
             ldb_k=4 * Co, ldb_n=1, ldc=4 * Co)
    bc = int(add is not None and add.shape[0] == 1 and B > 1)
    from ._lib import call
    call("s2h_convt2_ln_gelu", ops.dt(x), B, H, W, Co, ops.ptr(Y), ops.ptr(mod.bias.detach()), ops.ptr(add), bc,
         ops.ptr(ln.weight.detach()), ops.ptr(ln.bias.detach()), float(ln.eps), ops.ptr(pre), ops.ptr(y),
         ops.ptr(mean), ops.ptr(rstd), ops.ptr(post), ops.stream())
    return post


def point_embed(tape: FrameTape, pe, labels, dtype, tables):
    """PromptEncoder point embeddings (per-frame constant clicks + learned label embeddings)"""
    op, first = tape._begin("point_embed", [], _point_embed_bw, {"tables": tables})
    R, D = pe.shape[0] * pe.shape[1], pe.shape[2]
    table = torch.cat([p._s2h_compute.reshape(1, -1) for p in tables], 0).contiguous() if first else \
        op.attrs["table"]
    vid, out = tape._out(0, pe.shape, dtype)
    lab = tape._aux("labels", (R,), labels.dtype)
    if labels.dtype == torch.int32 and labels.is_contiguous():  # the kernel copies them beside the embedding
        ops.point_embed(pe.reshape(R, D), labels.reshape(R), table, out.view(R, D), labels_out=lab)
    else:
        ops.point_embed(pe.reshape(R, D), labels.reshape(R), table, out.view(R, D))
        lab.copy_(labels.reshape(R))
    if first:
        op.attrs["table"] = table
        op.attrs["D"] = D
    tape._finish(op, [vid], any(_grad_of(p) is not None for p in tables))
    return out


def _point_embed_bw(tape, op, gys):
    (g,) = gys
    D = op.attrs["D"]
    labels = tape.stores[("aux", op.idx, "labels")].buf
    gps = [_grad_of(p) for p in op.attrs["tables"]]
    n = len(gps)
    if n == 5 and all(gp is not None and gp.dtype == torch.float32 and gp.is_contiguous() and gp.numel() == D
                      for gp in gps):
        # accumulate straight into the label embeddings' arena gradients (no table, no adds)
        ops.point_embed_bwd_rows(labels, g.contiguous().view(-1, D), [gp.view(-1) for gp in gps])
        return []
    dtable = torch.zeros(n, D, device=g.device)
    ops.point_embed_bwd(labels, g.contiguous().view(-1, D), dtable)
    for i, gp in enumerate(gps):
        if gp is not None:
            ops.add(gp.view(-1), dtable[i], out=gp.view(-1))
    return []


# ---------------------------------------------------------------- two-way decoder, token side
def dec_tok_ok(x, blk, mlp_dim=2048):
    """the fused token-side launches (csrc/decoder_tok.hip) apply: bf16 tokens [B, T <= 16, 256], 8-head
    self-attention, 128-wide cross-attentions, a 256 -> 2048 -> 256 ReLU MLP, no dropout"""
    sa, t2i, i2t = blk.self_attn, blk.cross_attn_token_to_image, blk.cross_attn_image_to_token
    fc1, fc2 = blk.mlp.layers[0], blk.mlp.layers[-1]
    return (x.dtype == torch.bfloat16 and x.dim() == 3 and x.shape[1] <= 16 and x.shape[2] == 256
            and sa.num_heads == 8 and sa.internal_dim == 256 and t2i.internal_dim == 128
            and i2t.internal_dim == 128 and len(blk.mlp.layers) == 2 and blk.mlp.act == "relu"
            and not blk.mlp.sigmoid_output and fc1.out_features == mlp_dim and fc2.in_features == mlp_dim
            and sa.dropout_p == 0 and t2i.dropout_p == 0 and i2t.dropout_p == 0)


def _p(t):
    return t.data_ptr() if t is not None else None


def dec_self(tape: FrameTape, x, pe, sa, norm1, qc, skip):
    """The first half of a TwoWayAttentionBlock's token side (transformer.py:163-170): [q = x + pe] ->
    self-attention -> out-projection (+ x) -> norm1 -> x1; qt = x1 + pe -> token -> image q projection.
    Recorded as exactly those tape ops (so their backward is the usual one), computed by ONE
    s2h_dec_self launch.  Returns (x1, qq)."""
    from ._lib import call
    qa = None if skip else add(tape, x, pe, 1.0, 1.0, _compute=False)
    qin = x if skip else qa
    qs = linear(tape, qin, sa.q_proj, _compute=False)
    ks = linear(tape, qin, sa.k_proj, _compute=False)
    vs = linear(tape, x, sa.v_proj, _compute=False)
    B, L, C = qs.shape
    h = sa.num_heads
    scale = 1.0 / math.sqrt(C // h)
    os_, lse = attention(tape, qs.view(B, L, h, C // h), ks.view(B, L, h, C // h), vs.view(B, L, h, C // h), scale,
                         0.0, _compute=False)
    y1 = linear(tape, os_.reshape(B, L, C), sa.out_proj, residual=None if skip else x, _compute=False)
    x1, m1, r1 = layer_norm(tape, y1, norm1, norm1.eps, _compute=False)
    qt = add(tape, x1, pe, 1.0, 1.0, _compute=False)
    qq = linear(tape, qt, qc, _compute=False)
    w = lambda m: (_p(m.compute_weight()), _p(m.compute_bias()))  # noqa: E731
    call("s2h_dec_self", B * L, L, int(skip), float(scale), _p(x), _p(pe), *w(sa.q_proj), *w(sa.k_proj),
         *w(sa.v_proj), *w(sa.out_proj), _p(norm1.weight.detach()), _p(norm1.bias.detach()), float(norm1.eps),
         *w(qc), _p(qa), _p(qs), _p(ks), _p(vs), _p(os_), _p(lse), _p(y1), _p(x1), _p(m1), _p(r1), _p(qt), _p(qq),
         ops.stream())
    return x1, qq


def dec_post(tape: FrameTape, ot, x1, pe, out_proj, norm2, mlp, norm3, ki_mod, vi_mod, qf_mod=None):
    """The second half's token side (transformer.py:170-173): out-projection of the token -> image
    attention (+ x1) -> norm2 (one s2h_dec_post_a launch), the MLP's two GEMMs as usual, norm3 -> x3,
    q2 = x3 + pe -> the image -> token k / v projections, with qf_mod (the last block) also
    TwoWayTransformer's final q = x3 + pe and its projection (:194-196) (one s2h_dec_post_b launch).
    Recorded as those tape ops.  Returns (x3, ki, vi, qqf)."""
    from ._lib import call
    fc1, fc2 = mlp.layers[0], mlp.layers[-1]
    y2 = linear(tape, ot, out_proj, residual=x1, _compute=False)
    x2, m2, r2 = layer_norm(tape, y2, norm2, norm2.eps, _compute=False)
    B, L, C = x2.shape
    w = lambda m: (_p(m.compute_weight()), _p(m.compute_bias())) if m is not None else (None, None)  # noqa: E731
    call("s2h_dec_post_a", B * L, L, _p(ot), _p(x1), *w(out_proj), _p(norm2.weight.detach()),
         _p(norm2.bias.detach()), float(norm2.eps), _p(y2), _p(x2), _p(m2), _p(r2), ops.stream())
    y3 = linear(tape, linear(tape, x2, fc1, act="relu"), fc2, residual=x2)
    x3, m3, r3 = layer_norm(tape, y3, norm3, norm3.eps, _compute=False)
    q2 = add(tape, x3, pe, 1.0, 1.0, _compute=False)
    ki = linear(tape, q2, ki_mod, _compute=False)
    vi = linear(tape, x3, vi_mod, _compute=False)
    qfa = qqf = None
    if qf_mod is not None:
        qfa = add(tape, x3, pe, 1.0, 1.0, _compute=False)
        qqf = linear(tape, qfa, qf_mod, _compute=False)
    call("s2h_dec_post_b", B * L, L, int(qf_mod is not None), _p(y3), _p(pe), _p(norm3.weight.detach()),
         _p(norm3.bias.detach()), float(norm3.eps), *w(ki_mod), *w(vi_mod), *w(qf_mod), _p(x3), _p(m3), _p(r3),
         _p(q2), _p(ki), _p(vi), _p(qfa), _p(qqf), ops.stream())
    return x3, ki, vi, qqf


def dec_final(tape: FrameTape, of, x3, out_proj, norm):
    """TwoWayTransformer's final token side (transformer.py:196-197): out-projection (+ x3) -> norm,
    recorded as those two tape ops, one s2h_dec_final launch"""
    from ._lib import call
    y = linear(tape, of, out_proj, residual=x3, _compute=False)
    hs, m, r = layer_norm(tape, y, norm, norm.eps, _compute=False)
    B, L, C = x3.shape
    call("s2h_dec_final", B * L, L, _p(of), _p(x3), _p(out_proj.compute_weight()), _p(out_proj.compute_bias()),
         _p(norm.weight.detach()), _p(norm.bias.detach()), float(norm.eps), _p(y), _p(hs), _p(m), _p(r), ops.stream())
    return hs


def decoder_tokens(tape: FrameTape, sparse, dtype, params):
    """cat(obj_score_token, iou_token, mask_tokens) over objects + the sparse prompt rows"""
    op, first = tape._begin("tokens", [sparse], _tokens_bw, {"params": params})
    O, Ns, C = sparse.shape
    head = torch.cat([p._s2h_compute.reshape(-1, C) for p in params], 0) if first else op.attrs["head"]
    nh = head.shape[0]
    vid, out = tape._out(0, (O, nh + Ns, C), dtype)
    # the learned tokens (broadcast over the objects: source pitch 0) and the prompt rows, one launch
    ops.copy_segments([(head.unsqueeze(0).expand(O, -1, -1), out[:, :nh]), (sparse, out[:, nh:])])
    if first:
        op.attrs.update(head=head, nh=nh, Ns=Ns, C=C, O=O)
    tape._finish(op, [vid], any(op.needs) or any(_grad_of(p) is not None for p in params))
    return out


def _tokens_bw(tape, op, gys):
    (g,) = gys
    a = op.attrs
    F, O, nh, Ns, C = tape.F, a["O"], a["nh"], a["Ns"], a["C"]
    g3 = g.contiguous().view(F * O, nh + Ns, C)
    r = 0
    for p in a["params"]:
        gp = _grad_of(p)
        n = p.numel() // C
        if gp is not None:
            for j in range(n):
                ops.colsum(g3[:, r + j], gp.view(-1, C)[j], accumulate=True)
        r += n
    dsp = g3[:, nh:].contiguous().view(-1) if op.needs[0] else None
    return [dsp]


def memory_pos(tape: FrameTape, tpos_p, obj_pos, spatial_pos, tpos_idx, L, dtype, obj_rep=1):
    """memory positional table of this frame (sam2_base.py:597-674): spatial pos +
    maskmem_tpos_enc[tpos_idx[j]] per memory slot, then the object-pointer rows (constant; obj_rep > 1:
    one row per pointer, written into its obj_rep rows -- the repeat_interleave -- by one batched copy)"""
    op, first = tape._begin("memory_pos", [], _mpos_bw, {"tpos_p": tpos_p, "L": L})
    n = len(tpos_idx)
    Dm = spatial_pos.shape[-1]
    M = n * L + (obj_pos.shape[0] * obj_rep if obj_pos is not None else 0)
    tpos = tpos_p._s2h_compute.reshape(-1, Dm)
    if tpos.dtype != dtype:
        tpos = ops.cast(tpos.contiguous(), dtype)
    vid, out = tape._out(0, (M, Dm), dtype, tape.mem_rows)
    sp = spatial_pos.reshape(-1, Dm)
    if 0 < n <= 16 and sp.shape[0] == L and sp.is_contiguous() and tpos.is_contiguous():
        ops.memory_pos(sp, tpos, tpos_idx, out[:n * L])  # every slot in one launch
    else:
        for j, ti in enumerate(tpos_idx):
            ops.add_bcast(spatial_pos, tpos[ti], out=out[j * L:(j + 1) * L])
    if obj_pos is not None and obj_rep > 1:
        dst = out[n * L:].view(obj_pos.shape[0], obj_rep, Dm)
        ops.copy_segments([(obj_pos, dst[:, j]) for j in range(obj_rep)])
    elif obj_pos is not None:
        out[n * L:].copy_(obj_pos)
    tape._fattr(op, "tpos_idx", list(tpos_idx))
    tape._finish(op, [vid], _grad_of(tpos_p) is not None)
    return out


def _mpos_bw(tape, op, gys):
    (g,) = gys
    gt = _grad_of(op.attrs["tpos_p"])
    if gt is None:
        return []
    st = tape.st(op.outs[0])
    L = op.attrs["L"]
    Dm = st.shape0[-1]
    gt2 = gt.view(-1, Dm)
    segs = [((st.offsets[f] // Dm) + j * L, ti) for f in range(tape.F) for j, ti in enumerate(op.fattrs["tpos_idx"][f])]
    if 0 < len(segs) <= 64 and g.is_contiguous() and gt2.is_contiguous() and all(o % Dm == 0 for o in st.offsets):
        # every slot of every frame in one segmented column-sum launch
        ops.colsum_seg(g.view(-1, Dm), L, [o for o, _ in segs], [t for _, t in segs], gt2)
        return []
    for f in range(tape.F):
        gf = g[st.offsets[f]:st.offsets[f] + st.numels[f]].view(-1, Dm)
        for j, ti in enumerate(op.fattrs["tpos_idx"][f]):
            ops.colsum(gf[j * L:(j + 1) * L], gt2[ti], accumulate=True)
    return []
