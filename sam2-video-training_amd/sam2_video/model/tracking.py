"""Frame-batched training of the tracking loop (reference sam2model.py:266-401).

The forward stays sequential (frame t reads the bank frames < t wrote) and runs the same module
code as always; two FrameTapes (kernels/frametape.py) record it -- the memory attention of frames
1..T-1 and the SAM heads (prompt encoder + mask decoder + output head) of every frame that takes a
gradient -- with each op's saved tensors written into frame-stacked buffers.  One autograd node
(_TrackFn) then stands for the whole loop: its backward runs the SAM-heads tape once over all
frames, hands the gradient of the memory-conditioned features to the memory-attention tape, runs
that once over all frames, and returns the gradients of the backbone features (feats, high-res
s0 / s1).  Weight gradients go straight into the arena.  The memory encoder, object pointers and
bank writes stay outside the tapes (no gradient reaches them, sam2model.py:340-358).
"""
from __future__ import annotations

import torch

from ..kernels import functional as FN
from ..kernels import ops
from ..kernels.frametape import FrameTape, recording


class FrameTracker:
    """prompt_shapes: per frame, the shape of its sparse prompt (frames whose SAM heads see a
    different prompt size -- a box prompt on frame 0 -- record into a tape of their own)"""

    def __init__(self, model, T, O, feats, s0, s1, mask_mode, prompt_shapes=None):
        self.m = model
        self.T, self.O = T, O
        self.feats, self.s0, self.s1 = feats, s0, s1
        L, C = feats.shape[1], feats.shape[2]
        self.L, self.C = L, C
        dev = feats.device
        self.mask_mode = mask_mode
        self.dec_frames = [t for t in range(T) if not (t == 0 and mask_mode)]
        self.ma = (FrameTape(T - 1, dev, mem_rows=model._bank_rows(T, L, C), name="memory_attention")
                   if T > 1 else None)
        # SAM-heads tapes, one per prompt shape (frames in order)
        groups = {}
        for t in self.dec_frames:
            key = tuple(prompt_shapes[t]) if prompt_shapes is not None else ()
            groups.setdefault(key, []).append(t)
        self.decs = []  # [(tape, frames)]
        self.dec_of = {}  # t -> (group index, position)
        for gi, frames in enumerate(groups.values()):
            self.decs.append((FrameTape(len(frames), dev, name=f"sam_heads{gi}"), frames))
            for j, t in enumerate(frames):
                self.dec_of[t] = (gi, j)
        self.vids = [None] * len(self.decs)
        self.pix0 = None
        self.outs = {}  # t -> (high, ious)

    # ------------------------------------------------------------------ forward hooks
    def memory_conditioned(self, t, feat_t, pos, output_dict):
        m = self.m
        if t == 0:  # feat + no_mem_embed (sam2_base.py:680-684); its gradient is routed by hand
            with torch.no_grad():
                self.pix0 = m._prepare_memory_conditioned_features(0, True, feat_t, pos, self.T, output_dict, self.O)
            return self.pix0
        tp = self.ma
        tp.begin_frame()
        with recording(tp):
            f_in = tp.input("feat", feat_t, requires_grad=self.feats.requires_grad, stacked=(self.feats.detach(), 1))
            pix = m._prepare_memory_conditioned_features(t, False, f_in, pos, self.T, output_dict, self.O, tape=tp)
            if tp.f == 0:
                self.ma_out = tp.out_vid(pix)
        tp.end_frame()
        return pix

    def sam_heads(self, t, pix, prompt, s0t, s1t):
        gi, _ = self.dec_of[t]
        tp, frames = self.decs[gi]
        # the high-res features of consecutive frames are already stacked: alias, do not copy
        run = frames == list(range(frames[0], frames[0] + len(frames)))
        tp.begin_frame()
        with recording(tp):
            p_in = tp.input("pix", pix)
            s0_in = tp.input("s0", s0t, requires_grad=self.s0.requires_grad,
                             stacked=(self.s0.detach(), frames[0]) if run else None)
            s1_in = tp.input("s1", s1t, requires_grad=self.s1.requires_grad,
                             stacked=(self.s1.detach(), frames[0]) if run else None)
            low, high, ious, ptr, score = self.m._forward_sam_heads(p_in, prompt, (s0_in, s1_in), self.O)
            if tp.f == 0:
                self.vids[gi] = (tp.out_vid(high), tp.out_vid(ious))
        tp.end_frame()
        self.outs[t] = (high, ious)
        return low, high, ious, ptr, score

    # ------------------------------------------------------------------ autograd
    def finish(self):
        """connect the recorded loop to autograd: returns {t: (high, ious)} with grad_fn"""
        anchor = None
        for p in self.m.parameters():
            if p.requires_grad and getattr(p, "_s2h_grad", None) is not None:
                anchor = p
                break
        if anchor is None and not (self.feats.requires_grad or self.s0.requires_grad or self.s1.requires_grad):
            return self.outs
        flat = []
        for t in self.dec_frames:
            flat += list(self.outs[t])
        res = _TrackFn.apply(self, self.feats, self.s0, self.s1, anchor, *flat)
        out = dict(self.outs)
        for j, t in enumerate(self.dec_frames):
            out[t] = (res[2 * j], res[2 * j + 1])
        return out

    def backward(self, grads):
        T, O, L, C = self.T, self.O, self.L, self.C
        pix_n = O * L * C
        gpos = {t: j for j, t in enumerate(self.dec_frames)}  # position of frame t in `grads`
        dev = self.feats.device
        dpix = {}  # t -> flat d(pix) (views into the tapes' stacked gradients)
        dhr = {"s0": {}, "s1": {}}
        for gi, (tp, frames) in enumerate(self.decs):
            vh, vi = self.vids[gi]
            hs, is_ = tp.st(vh), tp.st(vi)
            gh = torch.empty(hs.buf.numel(), device=dev, dtype=hs.dtype)
            gio = torch.empty(is_.buf.numel(), device=dev, dtype=is_.dtype)
            pairs = []
            for j, t in enumerate(frames):
                for g, st, dst in ((grads[2 * gpos[t]], hs, gh), (grads[2 * gpos[t] + 1], is_, gio)):
                    d = dst[st.offsets[j]:st.offsets[j] + st.numels[j]]
                    if g is None:
                        d.zero_()
                    else:
                        pairs.append((g.reshape(-1), d))
            ops.copy_segments(pairs)
            din = tp.backward({vh: gh, vi: gio})
            for j, t in enumerate(frames):
                if din.get("pix") is not None:
                    dpix[t] = din["pix"][j * pix_n:(j + 1) * pix_n]
                for key in ("s0", "s1"):
                    g = din.get(key)
                    if g is not None:
                        per = g.numel() // len(frames)
                        dhr[key][t] = g[j * per:(j + 1) * per]
        dfeats = ds0 = ds1 = None
        if self.feats.requires_grad:
            dfeats = torch.zeros(T, L, C, device=dev, dtype=self.feats.dtype)
        if 0 in dpix and not self.mask_mode:  # frame 0: pix0 = expand(feat0 + no_mem_embed)
            d0 = dpix[0].view(O, L * C)
            if dfeats is not None:
                ops.sum_outer(d0, dfeats[0].view(-1))
            gm = FN._grad_of(self.m.no_mem_embed)
            if gm is not None:
                ops.colsum(d0.reshape(O * L, C), gm.view(-1), accumulate=True)
        have = [t in dpix for t in range(1, T)]
        if self.ma is not None and any(have) and not all(have):
            # every SAM-heads tape returns its pix gradient (zeros for unsupervised frames), so a
            # partial set means a broken tape -- never drop the memory-attention backward silently
            raise RuntimeError(f"memory-attention backward: pix gradients for frames "
                               f"{[t for t, h in zip(range(1, T), have) if h]} only (expected 1..{T - 1})")
        if self.ma is not None and have and all(have):
            # frames 1..T-1 stacked in order for the memory-attention tape (one copy unless a
            # single SAM-heads tape already holds them contiguously)
            g1 = dpix[1]
            es = g1.element_size()
            if all(dpix[t].data_ptr() == g1.data_ptr() + (t - 1) * pix_n * es for t in range(1, T)):
                gma = torch.as_strided(g1, ((T - 1) * pix_n,), (1,))
            else:
                gma = torch.cat([dpix[t] for t in range(1, T)])
            dma = self.ma.backward({self.ma_out: gma})
            if dfeats is not None and dma.get("feat") is not None:
                ops.add(dma["feat"], None, out=dfeats[1:].reshape(-1))
        for key, src in (("s0", self.s0), ("s1", self.s1)):
            if not src.requires_grad or not dhr[key]:
                continue
            full = torch.zeros(src.shape, device=dev, dtype=src.dtype)
            per = full[0].numel()
            ops.copy_segments([(g.reshape(-1), full.view(T, per)[t]) for t, g in dhr[key].items()])
            if key == "s0":
                ds0 = full
            else:
                ds1 = full
        return dfeats, ds0, ds1


class _TrackFn(torch.autograd.Function):
    """the whole tracking loop as one autograd node (forward already ran; backward batched)"""

    @staticmethod
    def forward(ctx, tracker, feats, s0, s1, anchor, *outs):
        ctx.tracker = tracker
        ctx.shapes = (feats.requires_grad, s0.requires_grad, s1.requires_grad)
        return tuple(o.view_as(o) for o in outs)

    @staticmethod
    def backward(ctx, *grads):
        dfeats, ds0, ds1 = ctx.tracker.backward(grads)
        rf, r0, r1 = ctx.shapes
        n = len(grads)
        return (None, dfeats if rf else None, ds0 if r0 else None, ds1 if r1 else None, None) + (None,) * n
