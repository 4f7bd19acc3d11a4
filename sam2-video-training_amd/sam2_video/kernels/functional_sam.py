"""SAM2-specific autograd functions over libsam2hip kernels: Hiera windowed
positional embedding (bicubic resize as two GEMMs), transposed-conv upscaling,
hypernetwork mask product, point-prompt embedding, memory-bank positional
encodings, category merge and the fused focal/Dice/IoU loss."""
from __future__ import annotations

import math
from functools import lru_cache

import numpy as np
import torch

from . import frametape as _ft
from . import ops
from .functional import _grad_of


# ------------------------------------------------- bicubic resize matrices
@lru_cache(maxsize=None)
def _bicubic_matrix_np(n_in: int, n_out: int):
    """PyTorch upsample_bicubic2d (align_corners=False, A=-0.75, clamped taps) as a matrix [n_out, n_in]."""
    A = -0.75
    scale = n_in / n_out
    M = np.zeros((n_out, n_in), np.float64)

    def c1(x):
        return ((A + 2) * x - (A + 3)) * x * x + 1

    def c2(x):
        return ((A * x - 5 * A) * x + 8 * A) * x - 4 * A

    for o in range(n_out):
        real = scale * (o + 0.5) - 0.5
        i0 = math.floor(real)
        t = real - i0
        ws = [c2(t + 1), c1(t), c1(1 - t), c2(2 - t)]
        for k in range(4):
            idx = min(max(i0 - 1 + k, 0), n_in - 1)
            M[o, idx] += ws[k]
    return M


@lru_cache(maxsize=None)
def _aa_bilinear_matrix_np(n_in: int, n_out: int):
    """PyTorch's antialiased bilinear resize (F.interpolate(mode="bilinear", antialias=True,
    align_corners=False), the _upsample_bilinear2d_aa weights) as a matrix [n_out, n_in]: a
    triangle filter of half-width `scale` when downsampling, normalised per output pixel."""
    scale = n_in / n_out
    support = scale if scale >= 1.0 else 1.0
    invscale = 1.0 / scale if scale >= 1.0 else 1.0
    M = np.zeros((n_out, n_in), np.float64)
    for i in range(n_out):
        center = scale * (i + 0.5)
        xmin = max(int(center - support + 0.5), 0)
        xsize = min(int(center + support + 0.5), n_in) - xmin
        ws = [max(0.0, 1.0 - abs((j + xmin - center + 0.5) * invscale)) for j in range(xsize)]
        tot = sum(ws)
        for j, wv in enumerate(ws):
            M[i, xmin + j] = wv / tot if tot != 0 else wv
    return M


_DEV_CACHE = {}


def aa_bilinear_matrix(n_in, n_out, device):
    key = ("aa", n_in, n_out, str(device))
    t = _DEV_CACHE.get(key)
    if t is None:
        t = torch.from_numpy(_aa_bilinear_matrix_np(n_in, n_out)).float().to(device)
        _DEV_CACHE[key] = t
    return t


def aa_downsample(x, ho, wo):
    """[N, hi, wi] f32 -> [N, ho, wo]: antialiased bilinear resize as two fp32 GEMMs with the
    separable weight matrices (forward only: the mask-prompt output path, sam2_base.py:446-452)"""
    N, hi, wi = x.shape
    Ah, Aw = aa_bilinear_matrix(hi, ho, x.device), aa_bilinear_matrix(wi, wo, x.device)
    Y1 = torch.empty(N * hi, wo, device=x.device)
    # Y1 = X Aw^T  ([N*hi, wi] x [wi, wo])
    ops.gemm(x.reshape(N * hi, wi), Aw, Y1, M=N * hi, N=wo, K=wi, lda_m=wi, lda_k=1, ldb_k=1, ldb_n=wi, ldc=wo)
    out = torch.empty(N, ho, wo, device=x.device)
    # out[n] = Ah Y1[n]  ([ho, hi] x [hi, wo])
    ops.gemm(Ah, Y1, out, M=ho, N=wo, K=hi, lda_m=hi, lda_k=1, ldb_k=wo, ldb_n=1, ldc=wo, batch=N, sA=0,
             sB=hi * wo, sC=ho * wo)
    return out


def bicubic_matrix(n_in, n_out, device):
    key = (n_in, n_out, str(device))
    t = _DEV_CACHE.get(key)
    if t is None:
        t = torch.from_numpy(_bicubic_matrix_np(n_in, n_out)).float().to(device)
        _DEV_CACHE[key] = t
    return t


class _PosEmbed(torch.autograd.Function):
    """Hiera._get_pos_embed (hieradet.py:273-281): bicubic(pos_embed -> h x w) + tiled window embed, -> [h, w, C]"""

    @staticmethod
    def forward(ctx, pe, win, h, w, dtype):
        _, C, bh, bw = pe.shape
        dev = pe.device
        Ah, Aw = bicubic_matrix(bh, h, dev), bicubic_matrix(bw, w, dev)
        X = pe.detach().reshape(C * bh, bw)
        Y1 = torch.empty(C * bh, w, device=dev)
        ops.gemm(X, Aw, Y1, M=C * bh, N=w, K=bw, lda_m=bw, lda_k=1, ldb_k=1, ldb_n=bw, ldc=w)
        Y2 = torch.empty(C, h, w, device=dev)
        ops.gemm(Ah, Y1, Y2, M=h, N=w, K=bh, lda_m=bh, lda_k=1, ldb_k=w, ldb_n=1, ldc=w, batch=C, sA=0,
                 sB=bh * w, sC=h * w)
        out = torch.empty(h, w, C, device=dev, dtype=dtype)
        ops.pos_embed(Y2, win.detach()[0], h, w, out)
        ctx.dims = (C, bh, bw, h, w, win.shape[-1])
        ctx.pe_p, ctx.win_p = pe, win
        ctx.save_for_backward(Ah, Aw)
        return out

    @staticmethod
    def backward(ctx, dout):
        Ah, Aw = ctx.saved_tensors
        C, bh, bw, h, w, ws = ctx.dims
        dev = dout.device
        gpe, gwin = _grad_of(ctx.pe_p), _grad_of(ctx.win_p)
        if gpe is None and gwin is None:
            return None, None, None, None, None
        dY2 = torch.empty(C, h, w, device=dev)
        ops.pos_embed_bwd(dout.contiguous(), dY2, gwin.view(-1) if gwin is not None else None, ws)
        if gpe is not None:
            dY1 = torch.empty(C, bh, w, device=dev)
            # dY1[c] = Ah^T @ dY2[c]
            ops.gemm(Ah, dY2, dY1, M=bh, N=w, K=h, lda_m=1, lda_k=bh, ldb_k=w, ldb_n=1, ldc=w, batch=C, sA=0,
                     sB=h * w, sC=bh * w)
            # dX = dY1 @ Aw  -> accumulate into the pos_embed gradient
            ops.gemm(dY1.view(C * bh, w), Aw, gpe.view(C * bh, bw), M=C * bh, N=bw, K=w, lda_m=w, lda_k=1,
                     ldb_k=bw, ldb_n=1, ldc=bw, beta=1.0)
        return None, None, None, None, None


def hiera_pos_embed(pe_param, win_param, h, w, dtype):
    return _PosEmbed.apply(pe_param, win_param, int(h), int(w), dtype)


# -------------------------------------------------- ConvTranspose2d(2, 2)
class _ConvT2(torch.autograd.Function):
    """x [B, H, W, Ci] -> [B, 2H, 2W, Co] = convT(x) + bias (+ add, broadcast over B when add has 1 batch)"""

    @staticmethod
    def forward(ctx, x, wp, bp, mod, add):
        B, H, W, Ci = x.shape
        Co = mod.out_ch
        w = mod.compute_weight()
        Y = torch.empty(B * H * W, 4 * Co, device=x.device, dtype=x.dtype)
        ops.gemm(x.reshape(-1, Ci), w, Y, M=B * H * W, N=4 * Co, K=Ci, lda_m=Ci, lda_k=1, ldb_k=4 * Co,
                 ldb_n=1, ldc=4 * Co)
        if ops.convt2_direct() and Co % (16 // x.element_size()) == 0:  # scatter + bias + add, one launch
            out = ops.convt2_store(Y, B, H, W, Co, bias=bp.detach(), add=None if add is None else add.contiguous())
        else:
            out = ops.convt2_scatter(Y, B, H, W, Co, bias=bp.detach(), add=None)
            if add is not None:
                if add.shape[0] == B:
                    out = ops.add(out, add.contiguous())
                else:
                    out = ops.add_bcast(out, add.contiguous())
        ctx.mod = mod
        ctx.add_bcast = add is not None and add.shape[0] != B
        ctx.has_add = add is not None
        ctx.save_for_backward(x)
        return out

    @staticmethod
    def backward(ctx, dout):
        (x,) = ctx.saved_tensors
        mod = ctx.mod
        B, H, W, Ci = x.shape
        Co = mod.out_ch
        dout = dout.contiguous()
        dY = ops.convt2_gather(dout, B, H, W, Co)
        gw, gb = _grad_of(mod.weight), _grad_of(mod.bias)
        if gw is not None:
            # dW[ci, n] += sum_rows x[row, ci] dY[row, n]
            ops.gemm(x.reshape(-1, Ci), dY, gw.view(Ci, 4 * Co), M=Ci, N=4 * Co, K=B * H * W, lda_m=1, lda_k=Ci,
                     ldb_k=4 * Co, ldb_n=1, ldc=4 * Co, beta=1.0)
        if gb is not None:
            ops.colsum(dout.view(-1, Co), gb)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(x.shape, device=x.device, dtype=x.dtype)
            ops.gemm(dY, mod.compute_weight(), dx.view(-1, Ci), M=B * H * W, N=Ci, K=4 * Co, lda_m=4 * Co, lda_k=1,
                     ldb_k=1, ldb_n=4 * Co, ldc=Ci)
        dadd = None
        if ctx.has_add and ctx.needs_input_grad[4]:
            if ctx.add_bcast:
                dadd = torch.empty((1, *dout.shape[1:]), device=dout.device, dtype=dout.dtype)
                ops.sum_outer(dout, dadd.view(-1))
            else:
                dadd = dout
        return dx, None, None, None, dadd


def conv_transpose2x2(x, mod, add=None):
    T = _ft.active()
    if T is not None:
        return _ft.conv_transpose2x2(T, x, mod, add)
    return _ConvT2.apply(x, mod.weight, mod.bias, mod, add)


# ----------------------------------------------------- hypernetwork masks
class _HyperMask(torch.autograd.Function):
    """masks[o, p] = sum_c hyper[o, c] * up[o, p, c]   (mask_decoder.py:227-234, token 0 only)"""

    @staticmethod
    def forward(ctx, hyper, up):
        O, P, C = up.shape
        out = torch.empty(O, 1, P, device=up.device, dtype=up.dtype)
        h3 = hyper.contiguous().view(O, 1, C)
        ops.bmm(h3, up, out, trans_b=True)
        ctx.save_for_backward(h3, up)
        return out.view(O, P)

    @staticmethod
    def backward(ctx, g):
        h3, up = ctx.saved_tensors
        O, P, C = up.shape
        g3 = g.contiguous().view(O, 1, P)
        dh = dup = None
        if ctx.needs_input_grad[0]:
            # a [1 x P] @ [P x C] reduction over P = 16k pixels per object: fp32 output lets the
            # GEMM split the reduction over workgroups (13 output tiles could not fill the chip)
            dh = torch.empty(O, 1, C, device=up.device, dtype=torch.float32)
            ops.bmm(g3, up, dh)
            dh = dh.view(O, C).to(up.dtype)
        if ctx.needs_input_grad[1]:
            dup = torch.empty(O, P, C, device=up.device, dtype=up.dtype)
            # dup[o] = g[o]^T (P x 1) @ hyper[o] (1 x C)
            ops.gemm(g3, h3, dup, M=P, N=C, K=1, lda_m=1, lda_k=P, ldb_k=C, ldb_n=1, ldc=C, batch=O, sA=P, sB=C,
                     sC=P * C)
        return dh, dup


def hyper_mask(hyper, up):
    T = _ft.active()
    if T is not None:
        return _ft.hyper_mask(T, hyper, up)
    return _HyperMask.apply(hyper, up)


# ------------------------------------------------------- point embeddings
class _PointEmbed(torch.autograd.Function):
    """PromptEncoder._embed_points label handling (prompt_encoder.py:79-121): the random-Fourier
    PE of the (host-side) clicks plus the learned label embeddings; pad/-1 clicks take
    not_a_point_embed only."""

    @staticmethod
    def forward(ctx, pe, labels, dtype, *tables):
        mods = tables  # not_a_point, pe0..pe3 parameters (compute copies are already in `dtype`)
        table = torch.cat([p._s2h_compute.reshape(1, -1) for p in mods], 0).contiguous()
        R, D = pe.shape[0] * pe.shape[1], pe.shape[2]
        out = torch.empty(pe.shape, device=pe.device, dtype=dtype)
        ops.point_embed(pe.view(R, D), labels.view(R), table, out.view(R, D))
        ctx.mods = mods
        ctx.save_for_backward(labels)
        return out

    @staticmethod
    def backward(ctx, g):
        (labels,) = ctx.saved_tensors
        g = g.contiguous()
        D = g.shape[-1]
        dtable = torch.zeros(5, D, device=g.device)
        ops.point_embed_bwd(labels.view(-1), g.view(-1, D), dtable)
        for i, p in enumerate(ctx.mods):
            gp = _grad_of(p)
            if gp is not None:
                ops.add(gp.view(-1), dtable[i], out=gp.view(-1))
        return (None, None, None) + tuple(None for _ in ctx.mods)


def point_embed(pe, labels, dtype, not_a_point, point_embeddings):
    tabs = [not_a_point.weight] + [e.weight for e in point_embeddings]
    T = _ft.active()
    if T is not None:
        return _ft.point_embed(T, pe, labels, dtype, tabs)
    return _PointEmbed.apply(pe, labels, dtype, *tabs)


# ------------------------------------------------------ memory positional
class _MemoryPos(torch.autograd.Function):
    """memory_pos of _prepare_memory_conditioned_features (sam2_base.py:597-674), batch-shared:
    rows of slot j = spatial pos + maskmem_tpos_enc[tpos_idx[j]], then the object-pointer rows."""

    @staticmethod
    def forward(ctx, tpos_p, obj_pos, spatial_pos, tpos_idx, L, dtype):
        n = len(tpos_idx)
        Dm = spatial_pos.shape[-1]
        tpos = tpos_p._s2h_compute.reshape(-1, Dm)
        if tpos.dtype != dtype:
            tpos = ops.cast(tpos.contiguous(), dtype)
        M = n * L + (obj_pos.shape[0] if obj_pos is not None else 0)
        out = torch.empty(M, Dm, device=spatial_pos.device, dtype=dtype)
        for j, ti in enumerate(tpos_idx):
            ops.add_bcast(spatial_pos, tpos[ti], out=out[j * L:(j + 1) * L])
        if obj_pos is not None:
            out[n * L:].copy_(obj_pos)
        ctx.tpos_p, ctx.tpos_idx, ctx.L = tpos_p, tpos_idx, L
        ctx.has_obj = obj_pos is not None
        return out

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        gt = _grad_of(ctx.tpos_p)
        L = ctx.L
        n = len(ctx.tpos_idx)
        if gt is not None:
            Dm = g.shape[-1]
            gt2 = gt.view(-1, Dm)
            for j, ti in enumerate(ctx.tpos_idx):
                ops.colsum(g[j * L:(j + 1) * L], gt2[ti], accumulate=True)
        dobj = g[n * L:] if (ctx.has_obj and ctx.needs_input_grad[1]) else None
        return None, dobj, None, None, None, None


def memory_pos(tpos_param, obj_pos, spatial_pos, tpos_idx, L, dtype, obj_rep=1):
    """obj_rep > 1: obj_pos holds one row per object pointer, each repeated obj_rep times"""
    T = _ft.active()
    if T is not None:
        return _ft.memory_pos(T, tpos_param, obj_pos, spatial_pos, list(tpos_idx), int(L), dtype, obj_rep)
    if obj_pos is not None and obj_rep > 1:
        obj_pos = obj_pos.repeat_interleave(obj_rep, dim=0)
    return _MemoryPos.apply(tpos_param, obj_pos, spatial_pos, list(tpos_idx), int(L), dtype)


# ------------------------------------------------------- category merge
class _MergeMasks(torch.autograd.Function):
    """pixelwise max over the objects of each category (masks.py:84-101)"""

    @staticmethod
    def forward(ctx, x, cat_off, cat_obj, obj_cat, ncat):
        O, P = x.shape[0], x[0].numel()
        out = torch.empty((ncat, *x.shape[1:]), device=x.device, dtype=torch.float32)
        arg = torch.empty(ncat, P, device=x.device, dtype=torch.int32)
        ops.group_max(x.reshape(O, P), cat_off, cat_obj, ncat, out.view(ncat, P), arg)
        ctx.save_for_backward(arg, obj_cat)
        ctx.shape = x.shape
        return out

    @staticmethod
    def backward(ctx, g):
        arg, obj_cat = ctx.saved_tensors
        O = ctx.shape[0]
        dx = torch.empty(ctx.shape, device=g.device, dtype=torch.float32)
        ops.group_max_bwd(g.contiguous().view(g.shape[0], -1), obj_cat, arg, dx.view(O, -1))
        return dx, None, None, None, None


class _MergeScores(torch.autograd.Function):
    """sigmoid-mass weighted mean per category (masks.py:70-82, 103-124); the weights come from
    the objects' high-res logits, so the backward also feeds d(weights) into those logits."""

    @staticmethod
    def forward(ctx, s, hr, cat_off, cat_obj, obj_cat, ncat):
        O = s.shape[0]
        hr2 = hr.detach().reshape(O, -1)
        stats = ops.mask_stats(hr2, None)
        out = torch.empty(ncat, s.shape[1], device=s.device, dtype=torch.float32)
        ops.group_wavg(s.contiguous(), stats, cat_off, cat_obj, ncat, out)
        ctx.save_for_backward(s, hr, stats, out, obj_cat, cat_off)
        return out

    @staticmethod
    def backward(ctx, g):
        s, hr, stats, out, obj_cat, cat_off = ctx.saved_tensors
        O = s.shape[0]
        ds = torch.empty_like(s)
        dw = torch.empty(O, device=s.device)
        ops.group_wavg_bwd(s.contiguous(), out, g.contiguous(), stats, obj_cat, cat_off, ds, dw)
        dhr = None
        if ctx.needs_input_grad[1]:
            dhr = torch.zeros(hr.shape, device=hr.device, dtype=torch.float32)
            ops.sigmoid_grad_axpy(hr.detach().reshape(O, -1), dw, dhr.view(O, -1))
        return ds, dhr, None, None, None, None


class _MergeMasksScores(torch.autograd.Function):
    """_MergeMasks of the high-res logits and _MergeScores weighted by the same logits as one node: the
    backward writes the max-merge gradient and adds the weights' sigmoid term into the same buffer
    (the sum autograd formed from two nodes, without its zero fill and add launches)"""

    @staticmethod
    def forward(ctx, hr, s, cat_off, cat_obj, obj_cat, ncat):
        O, P = hr.shape[0], hr[0].numel()
        out = torch.empty((ncat, *hr.shape[1:]), device=hr.device, dtype=torch.float32)
        arg = torch.empty(ncat, P, device=hr.device, dtype=torch.int32)
        ops.group_max(hr.reshape(O, P), cat_off, cat_obj, ncat, out.view(ncat, P), arg)
        stats = ops.mask_stats(hr.detach().reshape(O, -1), None)
        sout = torch.empty(ncat, s.shape[1], device=s.device, dtype=torch.float32)
        ops.group_wavg(s.contiguous(), stats, cat_off, cat_obj, ncat, sout)
        ctx.save_for_backward(arg, s, hr, stats, sout, obj_cat, cat_off)
        ctx.shape = hr.shape
        ctx.mark_non_differentiable(stats)
        return out, sout, stats

    @staticmethod
    def backward(ctx, g, gs, _gstats):
        arg, s, hr, stats, sout, obj_cat, cat_off = ctx.saved_tensors
        O = ctx.shape[0]
        dx = torch.empty(ctx.shape, device=hr.device, dtype=torch.float32)
        if g is None:
            dx.zero_()
        else:
            ops.group_max_bwd(g.contiguous().view(g.shape[0], -1), obj_cat, arg, dx.view(O, -1))
        ds = None
        if gs is not None:
            ds = torch.empty_like(s)
            dw = torch.empty(O, device=s.device)
            ops.group_wavg_bwd(s.contiguous(), sout, gs.contiguous(), stats, obj_cat, cat_off, ds, dw)
            ops.sigmoid_grad_axpy(hr.detach().reshape(O, -1), dw, dx.view(O, -1))
        return dx, ds, None, None, None, None


def merge_masks(x, groups):
    return _MergeMasks.apply(x, groups.cat_off, groups.cat_obj, groups.obj_cat, groups.ncat)


def merge_masks_scores(hr, s, groups):
    """(merge_masks(hr), merge_scores(s, hr), the per-object statistics of hr the weights come from) as
    one autograd node"""
    return _MergeMasksScores.apply(hr, s, groups.cat_off, groups.cat_obj, groups.obj_cat, groups.ncat)


def merge_scores_stats(s, stats, groups):
    """merge_scores(s, hr) without gradient, from hr's statistics already computed (merge_masks_scores)"""
    out = torch.empty(groups.ncat, s.shape[1], device=s.device, dtype=torch.float32)
    ops.group_wavg(s.contiguous(), stats, groups.cat_off, groups.cat_obj, groups.ncat, out)
    return out


def merge_scores(s, hr, groups):
    return _MergeScores.apply(s, hr, groups.cat_off, groups.cat_obj, groups.obj_cat, groups.ncat)


# ------------------------------------------------------------- the loss
class _FrameLoss(torch.autograd.Function):
    """one frame of MultiStepMultiMasksAndIous._update_losses (losses.py:143-238):
    returns [loss_mask, loss_dice, loss_iou, weighted total] for this frame."""

    @staticmethod
    def forward(ctx, logits, ious, tgt, valid, weights, inv_temp):
        N = logits.shape[0]
        x = logits.reshape(N, -1)
        P = x.shape[1]
        t = tgt.reshape(N, -1).view(torch.uint8)
        stats = ops.mask_stats(x, t, inv_temp)
        losses = torch.zeros(4, device=x.device)
        coef = torch.empty(N, 4, device=x.device)
        ops.mask_loss_finalize(stats, ious.reshape(N).contiguous(), valid, P, weights, 1.0, losses, coef)
        ctx.save_for_backward(x, t, coef)
        ctx.inv_temp = inv_temp
        ctx.shape = logits.shape
        return losses

    @staticmethod
    def backward(ctx, g):
        x, t, coef = ctx.saved_tensors
        # Gradients flow through the weighted total (entry 3; loss weights are folded into
        # coef); the per-term entries are logged values.  g[3] is read on device (no sync).
        dx = torch.empty_like(x)
        dious = torch.empty(x.shape[0], 1, device=x.device)
        ops.mask_loss_bwd(x, t, coef, ctx.inv_temp, dx, gtot=g.contiguous(), dious=dious)
        return dx.view(ctx.shape), dious, None, None, None, None


def frame_loss(logits, ious, tgt, valid, weights=(20.0, 1.0, 1.0), temperature=1.0):
    return _FrameLoss.apply(logits, ious, tgt, valid, tuple(float(w) for w in weights), 1.0 / float(temperature))


class _ClipLoss(torch.autograd.Function):
    """_FrameLoss of every frame of a clip summed (losses.py:111-121) as one node: the frames'
    finalize launches accumulate into one [4] buffer (the same fp32 additions in the same order as
    the per-frame buffers and their adds, without the per-frame zero fills and adds); the backward
    runs the per-frame gradient launches with the shared upstream gradient"""

    @staticmethod
    def forward(ctx, weights, inv_temp, n, *args):
        losses = None
        saved, shapes = [], []
        for f in range(n):
            logits, ious, tgt = args[3 * f:3 * f + 3]
            N = logits.shape[0]
            x = logits.reshape(N, -1)
            t = tgt.reshape(N, -1).view(torch.uint8)
            if losses is None:
                losses = torch.zeros(4, device=x.device)
            stats = ops.mask_stats(x, t, inv_temp)
            coef = torch.empty(N, 4, device=x.device)
            ops.mask_loss_finalize(stats, ious.reshape(N).contiguous(), None, x.shape[1], weights, 1.0, losses, coef)
            saved += [x, t, coef]
            shapes.append(logits.shape)
        ctx.save_for_backward(*saved)
        ctx.inv_temp, ctx.shapes, ctx.n = inv_temp, shapes, n
        return losses

    @staticmethod
    def backward(ctx, g):
        sv = ctx.saved_tensors
        gc = g.contiguous()
        grads = [None, None, None]
        for f in range(ctx.n):
            x, t, coef = sv[3 * f:3 * f + 3]
            dx = torch.empty_like(x)
            dious = torch.empty(x.shape[0], 1, device=x.device)
            ops.mask_loss_bwd(x, t, coef, ctx.inv_temp, dx, gtot=gc, dious=dious)
            grads += [dx.view(ctx.shapes[f]), dious, None]
        return tuple(grads)


def clip_loss(frames, weights=(20.0, 1.0, 1.0), temperature=1.0):
    """sum over frames of frame_loss(logits, ious, tgt, None) for frames = [(logits, ious, tgt), ...]"""
    flat = [t for fr in frames for t in fr]
    return _ClipLoss.apply(tuple(float(w) for w in weights), 1.0 / float(temperature), len(frames), *flat)


class _BCEFrame(torch.autograd.Function):
    """one frame of BCECategoryLoss (losses.py:306-366): BCE-with-logits over the categories with
    ground truth, reduced and scaled by 1/num_frames; accumulates into `acc` [1] f32"""

    @staticmethod
    def forward(ctx, logits, tgt, pos_weight, inv_temp, reduction, frame_scale):
        N = logits.shape[0]
        x = logits.reshape(N, -1)
        t = tgt.reshape(N, -1).view(torch.uint8)
        stats = ops.bce_stats(x, t, inv_temp, pos_weight)
        loss = torch.zeros(1, device=x.device)
        coef = torch.empty(N, device=x.device)
        ops.bce_finalize(stats, x.shape[1], reduction, frame_scale, loss, coef)
        ctx.save_for_backward(x, t, coef, pos_weight)
        ctx.inv_temp, ctx.shape = inv_temp, logits.shape
        return loss

    @staticmethod
    def backward(ctx, g):
        x, t, coef, pw = ctx.saved_tensors
        dx = torch.empty_like(x)
        ops.bce_bwd(x, t, ctx.inv_temp, pw, coef, dx, gtot=g.contiguous())
        return dx.view(ctx.shape), None, None, None, None, None


def bce_frame_loss(logits, tgt, pos_weight, temperature, reduction, frame_scale):
    return _BCEFrame.apply(logits, tgt, pos_weight, 1.0 / float(temperature), int(reduction), float(frame_scale))
