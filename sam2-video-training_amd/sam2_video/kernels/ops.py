"""Tensor-level launchers for libsam2hip (no autograd).  Every function launches
on torch's current HIP stream and returns its output tensor(s).

Conventions: activations are float32 (fp32-parity mode) or bfloat16 (compute
mode); norms' gamma/beta, biases, LSE/statistics and weight gradients are fp32.
"""
from __future__ import annotations

import contextlib
import math
import os

import torch

from ._lib import call, lib

F32, BF16 = 0, 1
ACT = {None: 0, "none": 0, "relu": 1, "gelu": 2, "sigmoid": 3}


def dt(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return F32
    if t.dtype == torch.bfloat16:
        return BF16
    raise TypeError(f"libsam2hip supports float32/bfloat16 activations, got {t.dtype}")


def ptr(t):
    return None if t is None else t.data_ptr()


def stream():
    return torch.cuda.current_stream().cuda_stream


_SIDE = {"on": os.environ.get("S2H_WGRAD_STREAM", "0") == "1", "streams": {}}


class SideWork:
    """Weight-gradient launches of one frame-tape backward on a second HIP stream, beside the
    input-gradient chain on the current one: a Linear's dW = dY^T X does not feed the next
    dgrad, so the two streams fill each other's ramp-up and tail (the step's GEMMs are short-K
    and latency-bound).  run(*reads) forks the side stream off the current one (an event) and
    keeps the tensors it reads alive; join() makes the current stream wait for everything
    forked and releases them -- the tape calls it before its gradients leave the backward, so
    nothing outside ever sees the second stream.  Graph capture records the fork / join as
    branches of the captured graph.  Opt-in (S2H_WGRAD_STREAM=1): on MI355X the second stream costs
    2.5 % of the bench step (59.5 vs 58.0 ms, profiles/r04_v4_wgrad_stream_ab.log) -- the weight
    gradients take CUs from the critical dgrad / attention-backward chain rather than filling idle
    ones (round 2 measured -4 % for the autograd form)."""

    def __init__(self):
        self.cur = self.ws = None
        _det_workspace_mode(not _SIDE["on"])
        if _SIDE["on"] and torch.cuda.is_available():
            self.cur = torch.cuda.current_stream()
            dev = self.cur.device
            ws = _SIDE["streams"].get(dev)
            if ws is None:
                ws = _SIDE["streams"][dev] = torch.cuda.Stream(dev)
            self.ws = ws
        self.refs = []
        self.used = False

    @contextlib.contextmanager
    def run(self, *reads):
        if self.ws is None:
            yield
            return
        self.ws.wait_stream(self.cur)
        with torch.cuda.stream(self.ws):
            yield
        self.refs.extend(t for t in reads if t is not None)
        self.used = True

    def join(self):
        if self.used:
            self.cur.wait_stream(self.ws)
        self.refs.clear()
        self.used = False


def _dev(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("libsam2hip kernels run on the GPU only (tensor on %s)" % t.device)


_RNG_OFFSET = {}


def rng_offset(device):
    """The device-resident uint64 dropout offset bound into libsam2hip (s2h_rng_bind): one per
    process, never freed (the library keeps its address).  Write it before a step (a fill
    kernel, no host sync) to draw fresh dropout masks, also on a replayed HIP graph."""
    t = _RNG_OFFSET.get("t")
    if t is None:
        t = torch.zeros(1, dtype=torch.int64, device=device)
        call("s2h_rng_bind", t.data_ptr())
        _RNG_OFFSET["t"] = t
    elif t.device.index != (torch.device(device).index if torch.device(device).index is not None
                            else torch.cuda.current_device()):
        raise RuntimeError(f"rng offset already bound on {t.device}, requested {device}")
    return t


# Workspace of the deterministic long-reduction weight-gradient GEMM (csrc/gemm_wgrad.hip): fp32
# partial tiles of <= ~256 (split, tile) workgroups x 256 KB plus the bias-gradient partials.  One per
# process, registered once, never freed (the library keeps its address); the GEMMs that use it are
# ordered on one stream -- with the opt-in weight-gradient side stream (S2H_WGRAD_STREAM) the library
# keeps the atomic split-K path instead (kmin 0).
WGRAD_WS_BYTES = 96 << 20
_WG_WS = {}


def _capturing():
    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()


def _persistent_alloc(what, n, dtype, device):
    """a buffer the library keeps the address of for the life of the process: never from a graph's
    private pool (a capture's allocations are released with the graph, the library would keep a
    dangling pointer) -- allocate it before the first capture (SAM2Model.load / StepRunner's eager
    warm-up do)"""
    if _capturing():
        raise RuntimeError(f"libsam2hip {what}: first use inside a HIP graph capture; allocate it before capturing "
                           f"(ops.{what}(device))")
    return torch.empty(n, dtype=dtype, device=device)


def _device_of(device):
    d = torch.device(device if device is not None else "cuda")
    if d.index is None:
        d = torch.device("cuda", torch.cuda.current_device())
    return d


WGRAD_KMIN = 4096  # csrc/gemm_wgrad.hip g_wg_kmin: reductions at least this long take the deterministic kernel


def _det_workspace_mode(on):
    """the library's deterministic-reduction workspace on (the default) or off: every user of it (the
    weight-gradient kernel, split-K partial tiles, fixed-order column sums) is ordered on ONE stream, so
    with the weight-gradient side stream (S2H_WGRAD_STREAM=1) they fall back to their atomic forms"""
    t = _WG_WS.get("t")
    if t is not None and _WG_WS.get("on", True) != on:
        call("s2h_wgrad_workspace", t.data_ptr(), WGRAD_WS_BYTES, WGRAD_KMIN if on else 0)
    _WG_WS["on"] = on


def wgrad_workspace(device=None):
    d = _device_of(device)
    t = _WG_WS.get("t")
    if t is None:
        t = _persistent_alloc("wgrad_workspace", WGRAD_WS_BYTES // 4, torch.float32, d)
        on = not _SIDE["on"]
        call("s2h_wgrad_workspace", t.data_ptr(), WGRAD_WS_BYTES, WGRAD_KMIN if on else 0)
        _WG_WS["t"] = t
        _WG_WS["on"] = on
    elif t.device != d:  # one registration per process: the library holds one address
        raise RuntimeError(f"wgrad workspace already registered on {t.device}, requested {d}")
    return t


# Deferred gradient sums (csrc/grad_defer.hip): inside the scope, the fixed-order second pass of the
# column reductions whose destination lies in `sink` (the gradient arena: LayerNorm gamma / beta, bias
# gradients) is recorded and run for all of them in a few launches when the scope closes.  The scope
# must enclose whole backward passes whose arena gradients nothing reads before it closes (the
# StepRunner's backward phases; the DDP all-reduce of a range is issued after its phase's scope).
# S2H_GRAD_DEFER=0 keeps the immediate second pass (A/B).
GRAD_DEFER_BYTES = 256 << 20
_DEFER = {"t": None, "depth": 0}


def grad_defer_enabled():
    return os.environ.get("S2H_GRAD_DEFER", "1") == "1"


@contextlib.contextmanager
def deferred_grad_sums(sink):
    if sink is None or not sink.is_cuda or _DEFER["depth"] > 0 or not grad_defer_enabled():
        _DEFER["depth"] += 1
        try:
            yield
        finally:
            _DEFER["depth"] -= 1
        return
    t = _DEFER["t"]
    if t is None or t.device != sink.device:
        t = _DEFER["t"] = _persistent_alloc("deferred_grad_sums", GRAD_DEFER_BYTES // 4, torch.float32, sink.device)
    call("s2h_grad_defer", t.data_ptr(), GRAD_DEFER_BYTES, sink.data_ptr(), sink.numel() * sink.element_size())
    _DEFER["depth"] += 1
    try:
        yield
    finally:
        _DEFER["depth"] -= 1
        try:
            call("s2h_grad_defer_flush", stream())
        finally:  # the scope ends even when the flush raised: later scopes must be able to register
            call("s2h_grad_defer_reset")


# ----------------------------------------------------------------- GEMM
def gemm(a, b, c, *, M, N, K, lda_m, lda_k, ldb_k, ldb_n, ldc, batch=1, sA=0, sB=0, sC=0,
         bias=None, bias_mode=1, residual=None, ldr=0, sR=0, aux=None, ldx=0, sX=0, aux_mode=0,
         cscale=None, drop_p=0.0, seed=0, alpha=1.0, beta=0.0, act=0, drop_idx0=0):
    _dev(a, b, c, bias, residual, aux)
    if bias is not None:
        assert bias.dtype == torch.float32 and bias.is_contiguous()
    if c.dtype == torch.float32 and K >= 512 and "t" not in _WG_WS:
        wgrad_workspace(c.device)
    call("s2h_gemm", dt(a), dt(c), batch, M, N, K,
         ptr(a), lda_m, lda_k, sA, ptr(b), ldb_k, ldb_n, sB, ptr(c), ldc, sC,
         ptr(bias), bias_mode, ptr(residual), ldr, sR, ptr(aux), ldx, sX, aux_mode,
         ptr(cscale), float(drop_p), int(seed) & (2**64 - 1), int(drop_idx0), float(alpha), float(beta), int(act),
         stream())
    return c


def _rows(x):
    assert x.stride(-1) == 1, "last dim must be contiguous"
    return x.numel() // x.shape[-1], x.shape[-1]


def linear(x, w, bias=None, act=None, out=None, pre=None, residual=None, out_dtype=None, cscale=None,
           drop_p=0.0, seed=0, drop_idx0=0):
    """out = drop(act(x @ w^T + bias) * cscale) (+ residual); optionally stores the pre-activation in `pre`."""
    x2 = x.reshape(-1, x.shape[-1])
    M, K = x2.shape
    N = w.shape[0]
    assert w.shape[1] == K and w.is_contiguous()
    if out is None:
        out = torch.empty(*x.shape[:-1], N, device=x.device, dtype=out_dtype or x.dtype)
    o2 = out.view(-1, N)
    r2 = residual.reshape(-1, N) if residual is not None else None
    p2 = pre.view(-1, N) if pre is not None else None
    gemm(x2, w, o2, M=M, N=N, K=K, lda_m=x2.stride(0), lda_k=1, ldb_k=1, ldb_n=K, ldc=N,
         bias=bias, residual=r2, ldr=N, aux=p2, ldx=N, aux_mode=1 if pre is not None else 0, act=ACT[act],
         cscale=cscale, drop_p=drop_p, seed=seed, drop_idx0=drop_idx0)
    return out


def rope_blocks(y2, rp, inverse=False):
    """in place axial RoPE of a [rows, N] matrix (C contiguous): rp = (cos, sin, L, nrot, period,
    ncol, dh) rotates, in every block of L rows, the rows < nrot in the columns < ncol (dh-wide
    heads, pairs (2i, 2i + 1))"""
    cos, sin, L, nrot, period, ncol, dh = rp
    rows, N = y2.shape
    assert rows % L == 0 and y2.stride(1) == 1
    ld = y2.stride(0)
    for c0 in range(0, ncol, dh):
        v = torch.as_strided(y2, (rows // L, L, dh), (L * ld, ld, 1), y2.storage_offset() + c0)
        rope(v, v, nrot, cos, sin, period, inverse)
    return y2


def linear_rope(x, w, bias, rp, out=None):
    """out = RoPE(x @ w^T + bias) (rope_blocks' layout): one GEMM with the rotation in its epilogue
    in bf16 (s2h_linear_rope), GEMM + in-place rotation in fp32"""
    x2 = x.reshape(-1, x.shape[-1])
    M, K = x2.shape
    N = w.shape[0]
    assert w.shape[1] == K and w.is_contiguous()
    if out is None:
        out = torch.empty(*x.shape[:-1], N, device=x.device, dtype=x.dtype)
    o2 = out.view(-1, N)
    cos, sin, L, nrot, period, ncol, dh = rp
    if x.dtype == torch.bfloat16 and x2.stride(1) == 1:
        _dev(x2, w, o2, bias)
        call("s2h_linear_rope", M, N, K, ptr(x2), x2.stride(0), ptr(w), w.stride(0), ptr(bias), ptr(o2), N, ptr(cos),
             ptr(sin), int(L), int(nrot), int(period), int(ncol), int(dh), stream())
        return out
    linear(x, w, bias, out=out)
    rope_blocks(o2, rp)
    return out


def linear_add_ln(x, w, bias, residual, gamma, beta, eps, drop_p=0.0, seed=0, drop_idx0=0, xsum=None, y=None,
                  mean=None, rstd=None):
    """xsum = residual + dropout(x @ w^T + bias), y = LN(xsum) (gamma, beta, eps), mean / rstd per row, in
    one launch (s2h_linear_add_ln; bf16, N = 128 or 256); returns (y, xsum, mean, rstd)"""
    x2 = x.reshape(-1, x.shape[-1])
    M, K = x2.shape
    N = w.shape[0]
    assert w.shape[1] == K and w.is_contiguous() and x2.stride(1) == 1 and x.dtype == torch.bfloat16
    shape = (*x.shape[:-1], N)
    xsum = torch.empty(shape, device=x.device, dtype=x.dtype) if xsum is None else xsum
    y = torch.empty(shape, device=x.device, dtype=x.dtype) if y is None else y
    mean = torch.empty(M, device=x.device, dtype=torch.float32) if mean is None else mean
    rstd = torch.empty(M, device=x.device, dtype=torch.float32) if rstd is None else rstd
    r2 = residual.reshape(-1, N) if residual is not None else None
    _dev(x2, w, bias, r2, xsum, y, gamma, beta, mean, rstd)
    call("s2h_linear_add_ln", M, N, K, ptr(x2), x2.stride(0), ptr(w), w.stride(0), ptr(bias), ptr(r2),
         r2.stride(0) if r2 is not None else 0, float(drop_p), int(seed) & (2**64 - 1), int(drop_idx0), ptr(xsum), N,
         ptr(gamma), ptr(beta), float(eps), ptr(y), N, ptr(mean), ptr(rstd), stream())
    return y, xsum, mean, rstd


def linear_dgrad(dy, w, dx=None, accumulate=False, pre=None, act=None, alpha=1.0, residual=None):
    """dx = alpha * dy @ w   (optionally * act'(pre) elementwise, fusing the previous layer's
    activation grad; for ReLU `pre` may be the previous layer's output, and alpha its 1/keep);
    accumulate: dx += ...; residual [rows, K] (same dtype, contiguous): dx = ... + residual (one
    rounding of the fp32 sum)"""
    dy2 = dy.reshape(-1, dy.shape[-1])
    M, N = dy2.shape
    K = w.shape[1]
    if dx is None:
        dx = torch.empty(*dy.shape[:-1], K, device=dy.device, dtype=dy.dtype)
    d2 = dx.view(-1, K)
    p2 = pre.reshape(-1, K) if pre is not None else None
    r2 = residual.view(-1, K) if residual is not None else None
    gemm(dy2, w, d2, M=M, N=K, K=N, lda_m=dy2.stride(0), lda_k=1, ldb_k=K, ldb_n=1, ldc=K,
         aux=p2, ldx=K, aux_mode=2 if pre is not None else 0, act=ACT[act] if pre is not None else 0,
         alpha=alpha, beta=1.0 if accumulate else 0.0, residual=r2, ldr=K if r2 is not None else 0)
    return dx


def ffn_bwd_dgrad_ok(dy, w2, w1, hid):
    """s2h_ffn_bwd_dgrad applies: bf16, d_model 256, hidden a multiple of 128, rows a multiple of 64,
    contiguous weights, unit-stride 16-B aligned rows"""
    if dy.dim() != 2 or hid.dim() != 2:
        return False
    R, H = hid.shape
    return (all(t.dtype == torch.bfloat16 for t in (dy, w2, w1, hid)) and dy.shape == (R, 256)
            and tuple(w2.shape) == (256, H) and tuple(w1.shape) == (H, 256) and H % 128 == 0 and R % 64 == 0
            and w2.is_contiguous() and w1.is_contiguous() and hid.is_contiguous() and dy.stride(1) == 1
            and dy.stride(0) % 8 == 0 and R * max(H, dy.stride(0)) < 2**31
            and all(t.data_ptr() % 16 == 0 for t in (dy, w2, w1, hid)))


def ffn_bwd_dgrad(dy, w2, w1, hid, alpha=1.0, dh=None, dx=None):
    """Memory-attention FFN backward, input-gradient side, in one launch (csrc/ffn.hip):
    dh = alpha * (dy @ w2) * [hid > 0] (linear1's pre-activation gradient) and dx = dh @ w1.
    dy [R, 256], w2 [256, H] (linear2.weight), w1 [H, 256] (linear1.weight), hid [R, H] (linear2's
    saved input).  Returns (dh, dx)."""
    assert ffn_bwd_dgrad_ok(dy, w2, w1, hid)
    R, H = hid.shape
    if dh is None:
        dh = torch.empty(R, H, device=dy.device, dtype=dy.dtype)
    if dx is None:
        dx = torch.empty(R, 256, device=dy.device, dtype=dy.dtype)
    _dev(dy, w2, w1, hid, dh, dx)
    call("s2h_ffn_bwd_dgrad", R, H, ptr(dy), dy.stride(0), ptr(w2), ptr(w1), ptr(hid), H, float(alpha), ptr(dh),
         dh.stride(0), ptr(dx), dx.stride(0), stream())
    return dh, dx


def ffn_fwd_ok(x, w1, b1, w2, b2):
    """s2h_ffn_fwd applies: bf16, d_model 256, hidden 1024 or 2048, rows a multiple of 64,
    contiguous 16-B aligned operands, fp32 biases"""
    if x.dim() != 2:
        return False
    R, C = x.shape
    H = w1.shape[0]
    return (x.dtype == torch.bfloat16 and w1.dtype == torch.bfloat16 and w2.dtype == torch.bfloat16
            and b1 is not None and b2 is not None and b1.dtype == torch.float32 and b2.dtype == torch.float32
            and C == 256 and tuple(w1.shape) == (H, 256) and tuple(w2.shape) == (256, H) and H in (1024, 2048)
            and R % 64 == 0 and R * max(H, x.stride(0)) < 2**31 and x.stride(1) == 1 and x.stride(0) % 8 == 0
            and all(t.is_contiguous() for t in (w1, w2, b1, b2))
            and all(t.data_ptr() % 16 == 0 for t in (x, w1, w2, b1, b2)))


def ffn_fwd(x, w1, b1, w2, b2, p=0.0, seed1=0, idx1=0, seed2=0, idx2=0, hid=None, y=None):
    """Memory-attention FFN forward in one launch (csrc/ffn.hip): hid = drop(relu(x w1^T + b1)),
    y = drop(hid w2^T + b2) with the GEMM epilogue's dropout hash (seed1 / idx1, seed2 / idx2).
    Returns (hid, y)."""
    assert ffn_fwd_ok(x, w1, b1, w2, b2)
    R = x.shape[0]
    H = w1.shape[0]
    if hid is None:
        hid = torch.empty(R, H, device=x.device, dtype=x.dtype)
    if y is None:
        y = torch.empty(R, 256, device=x.device, dtype=x.dtype)
    assert hid.is_contiguous() and y.is_contiguous()
    _dev(x, w1, b1, w2, b2, hid, y)
    call("s2h_ffn_fwd", R, H, ptr(x), x.stride(0), ptr(w1), ptr(b1), ptr(w2), ptr(b2), float(p),
         int(seed1) & (2**64 - 1), int(idx1), int(seed2) & (2**64 - 1), int(idx2), ptr(hid), H, ptr(y), 256, stream())
    return hid, y


def linear_dgrad_ln_bwd_ok(dy, w, x):
    """s2h_linear_dgrad_ln_bwd applies: bf16, LayerNorm width 128 / 256, 16-B aligned rows"""
    K = w.shape[1]
    return (dy.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.dtype == torch.bfloat16 and K in (128, 256)
            and w.is_contiguous() and dy.shape[-1] % 8 == 0 and dy.stride(-1) == 1 and x.is_contiguous()
            and all(t.data_ptr() % 16 == 0 for t in (dy, w, x)))


def linear_dgrad_ln_bwd(dy, w, x, gamma, mean, rstd, dres=None, dgamma=None, dbeta=None, alpha=1.0, dx=None):
    """dx = LN'(alpha * dy @ w) + dres for a LayerNorm (input x, gamma, saved mean / rstd) whose output
    feeds only the Linear with weight w; dgamma / dbeta += its weight gradients -- one full-row GEMM
    launch with the LayerNorm backward in the epilogue (+ the partial-row finalize)"""
    dy2 = dy.reshape(-1, dy.shape[-1])
    M, N = dy2.shape
    C = w.shape[1]
    x2 = x.reshape(-1, C)
    assert x2.shape[0] == M and w.shape[0] == N and mean.numel() >= M and rstd.numel() >= M
    if dx is None:
        dx = torch.empty(x.shape, device=dy.device, dtype=dy.dtype)
    d2 = dx.view(-1, C)
    r2 = dres.reshape(-1, C) if dres is not None else None
    if r2 is not None:
        assert r2.stride(1) == 1 and r2.dtype == dx.dtype
    part = None
    if dgamma is not None:
        nbytes = lib().s2h_linear_dgrad_ln_bwd_ws_bytes(M, C)
        part = torch.empty(max(nbytes // 4, 1), device=dy.device, dtype=torch.float32)
    _dev(dy2, w, x2, gamma, mean, rstd, r2, d2, dgamma, dbeta)
    call("s2h_linear_dgrad_ln_bwd", M, C, N, ptr(dy2), dy2.stride(0), ptr(w), w.stride(0), float(alpha), ptr(x2), C,
         ptr(gamma), ptr(mean), ptr(rstd), ptr(r2), r2.stride(0) if r2 is not None else 0, ptr(d2), C, ptr(part),
         ptr(dgamma), ptr(dbeta), stream())
    return dx


def mlp_heads(heads, outs=None, hidden=None, pre=None):
    """MLP heads in one launch (s2h_mlp_heads): heads = [(x [M, K0] bf16 rows, [W_l] bf16 [N_l, K_l],
    [b_l fp32 or None], act_last)] with the same M; ReLU between layers.  outs: optional [y] to write;
    hidden: optional [[h_l]] per head (each hidden layer's ReLU output, contiguous); pre: optional
    [pre-activation of the last layer or None] per head.  Returns [y]"""
    import ctypes
    n = len(heads)
    M = heads[0][0].shape[0]
    xs, lds, ws, bs, dims, nls, acts, ys, ldys = [], [], [], [], [], [], [], [], []
    hids, pres = [], []
    for hi, (x, wl, bl, act_last) in enumerate(heads):
        assert x.dtype == torch.bfloat16 and x.shape[0] == M and x.stride(1) == 1 and len(wl) <= 3
        y = outs[hi] if outs is not None else torch.empty(M, wl[-1].shape[0], device=x.device, dtype=x.dtype)
        assert y.shape == (M, wl[-1].shape[0]) and y.stride(1) == 1
        hl = hidden[hi] if hidden is not None else []
        for h, w in zip(hl, wl[:-1]):
            assert h.is_contiguous() and h.shape == (M, w.shape[0])
        hids += [ptr(h) for h in hl] + [None] * (2 - len(hl))
        pl = pre[hi] if pre is not None else None
        assert pl is None or (pl.is_contiguous() and pl.shape == y.shape)
        pres.append(ptr(pl))
        _dev(x, y, *wl, *[b for b in bl if b is not None])
        xs.append(ptr(x))
        lds.append(x.stride(0))
        d = [x.shape[1]] + [w.shape[0] for w in wl]
        for w, k in zip(wl, d[:-1]):
            assert w.is_contiguous() and w.dtype == torch.bfloat16 and w.shape[1] == k
        dims += d + [0] * (4 - len(d))
        ws += [ptr(w) for w in wl] + [None] * (3 - len(wl))
        bs += [ptr(b) for b in bl] + [None] * (3 - len(bl))
        nls.append(len(wl))
        acts.append(ACT[act_last])
        ys.append(y)
        ldys.append(y.stride(0))
    P = ctypes.c_void_p
    call("s2h_mlp_heads", n, M, (P * n)(*xs), (ctypes.c_int64 * n)(*lds), (P * (3 * n))(*ws),
         (P * (3 * n))(*bs), (ctypes.c_int * (4 * n))(*dims), (ctypes.c_int * n)(*nls), (ctypes.c_int * n)(*acts),
         (P * n)(*[ptr(y) for y in ys]), (ctypes.c_int64 * n)(*ldys),
         (P * (2 * n))(*hids) if hidden is not None else None, (P * n)(*pres) if pre is not None else None, stream())
    return ys


def linear_wgrad(dy, x, dw, accumulate=True, db=None):
    """dw (fp32 [N, K]) (+)= dy^T @ x;  db (fp32 [N], optional) (+)= dy summed over rows."""
    dy2 = dy.reshape(-1, dy.shape[-1])
    x2 = x.reshape(-1, x.shape[-1])
    M, N = dy2.shape
    K = x2.shape[1]
    assert dw.dtype == torch.float32 and dw.shape == (N, K) and dw.stride(1) == 1
    assert dy2.dtype == x2.dtype and dy2.stride(1) == 1 and x2.stride(1) == 1
    if db is not None:
        assert db.dtype == torch.float32 and db.numel() == N and db.is_contiguous()
    _dev(dy2, x2, dw, db)
    if M >= 512 and "t" not in _WG_WS:
        wgrad_workspace(dw.device)
    call("s2h_linear_wgrad", dt(dy2), M, N, K, ptr(dy2), dy2.stride(0), ptr(x2), x2.stride(0), ptr(dw), dw.stride(0),
         ptr(db), int(accumulate), stream())
    return dw


# ----------------------------------------------------------------- MX-fp8 (config 5)
class MX8:
    """An MX-fp8 (OCP MXFP8-E4M3) operand as s2h_mx8_quant writes it: `q` [rows, Kp] uint8 e4m3
    codes (Kp = k rounded up to 128, zero padded), `s` [Kp / 128, rows] int32 scale words (byte b
    of word (kt, r) = E8M0 exponent of the 32-block 4kt + b of row r), `k` the logical depth."""
    __slots__ = ("q", "s", "k")

    def __init__(self, q, s, k):
        self.q, self.s, self.k = q, s, k

    @property
    def rows(self):
        return self.q.shape[0]


def mx8_empty(rows, k, device):
    kp = (k + 127) // 128 * 128
    return MX8(torch.empty(rows, kp, dtype=torch.uint8, device=device),
               torch.empty(kp // 128, rows, dtype=torch.int32, device=device), k)


def mx8_quant(x, out=None, transpose=False):
    """MX-fp8 of the rows of 2-D `x` [rows, cols] (blocks along cols, cols contiguous), or with
    transpose=True of x^T ([cols, rows] -> blocks along x's rows: the dgrad operand of a weight)."""
    _dev(x)
    assert x.dim() == 2
    if transpose:
        assert x.stride(0) == 1 or x.is_contiguous()
        rows, cols = x.shape[1], x.shape[0]
        ld_row, ld_col = x.stride(1), x.stride(0)
    else:
        assert x.stride(1) == 1
        rows, cols = x.shape
        ld_row, ld_col = x.stride(0), 1
    if out is None:
        out = mx8_empty(rows, cols, x.device)
    assert out.q.shape[0] == rows and out.k == cols and out.s.shape[1] >= rows
    call("s2h_mx8_quant", rows, cols, dt(x), ptr(x), ld_row, ld_col, ptr(out.q), out.q.stride(0), ptr(out.s),
         out.s.stride(0), stream())
    return out


def gemm_mx8(a: MX8, b: MX8, c, *, bias=None, residual=None, aux=None, aux_mode=0, act=0, drop_p=0.0, seed=0,
             drop_idx0=0, alpha=1.0, beta=0.0):
    """c[M, N] = epilogue(alpha * A B^T) for MX-fp8 A [M, K] and B [N, K] (s2h_gemm_mx8)"""
    assert a.k == b.k and c.dim() == 2 and c.stride(1) == 1
    M, N = a.rows, b.rows
    assert c.shape == (M, N)
    _dev(a.q, b.q, c, bias, residual, aux)
    call("s2h_gemm_mx8", M, N, a.k, ptr(a.q), a.q.stride(0), ptr(a.s), a.s.stride(0), ptr(b.q), b.q.stride(0),
         ptr(b.s), b.s.stride(0), ptr(c), dt(c), c.stride(0), ptr(bias), ptr(residual),
         residual.stride(0) if residual is not None else 0, ptr(aux), aux.stride(0) if aux is not None else 0,
         aux_mode if aux is not None else 0, float(drop_p), int(seed) & (2**64 - 1), int(drop_idx0), float(alpha),
         float(beta), int(act), stream())
    return c


def linear_mx8(x, w8: MX8, bias=None, act=None, out=None, pre=None, residual=None, drop_p=0.0, seed=0, drop_idx0=0):
    """ops.linear with MX-fp8 operands: x (bf16) quantised here, w8 = the weight's MX-fp8 copy."""
    x2 = x.reshape(-1, x.shape[-1])
    N = w8.rows
    assert x2.shape[1] == w8.k
    if out is None:
        out = torch.empty(*x.shape[:-1], N, device=x.device, dtype=x.dtype)
    xq = mx8_quant(x2 if x2.stride(1) == 1 else x2.contiguous())
    gemm_mx8(xq, w8, out.view(-1, N), bias=bias, residual=residual.reshape(-1, N) if residual is not None else None,
             aux=pre.view(-1, N) if pre is not None else None, aux_mode=1 if pre is not None else 0, act=ACT[act],
             drop_p=drop_p, seed=seed, drop_idx0=drop_idx0)
    return out


def linear_dgrad_mx8(dy, wt8: MX8, dx=None, accumulate=False, pre=None, act=None, alpha=1.0):
    """ops.linear_dgrad with MX-fp8 operands: dy quantised along its N, wt8 = MX-fp8 of W^T [K, N]."""
    dy2 = dy.reshape(-1, dy.shape[-1])
    K = wt8.rows
    assert dy2.shape[1] == wt8.k
    if dx is None:
        dx = torch.empty(*dy.shape[:-1], K, device=dy.device, dtype=dy.dtype)
    dq = mx8_quant(dy2 if dy2.stride(1) == 1 else dy2.contiguous())
    gemm_mx8(dq, wt8, dx.view(-1, K), aux=pre.reshape(-1, K) if pre is not None else None,
             aux_mode=2 if pre is not None else 0, act=ACT[act] if pre is not None else 0, alpha=alpha,
             beta=1.0 if accumulate else 0.0)
    return dx


def bmm(a, b, out, *, trans_b=False, alpha=1.0, beta=0.0):
    """Batched out[i] = a[i] @ b[i] (or b[i]^T): a [Bt, M, K], b [Bt, K, N] / [Bt, N, K]."""
    Bt, M, K = a.shape
    if trans_b:
        N = b.shape[1]
        ldb_k, ldb_n = b.stride(2), b.stride(1)
    else:
        N = b.shape[2]
        ldb_k, ldb_n = b.stride(1), b.stride(2)
    gemm(a, b, out, M=M, N=N, K=K, lda_m=a.stride(1), lda_k=a.stride(2), ldb_k=ldb_k, ldb_n=ldb_n,
         ldc=out.stride(1), batch=Bt, sA=a.stride(0), sB=b.stride(0), sC=out.stride(0), alpha=alpha, beta=beta)
    return out


# ------------------------------------------------------------ attention
def _bhl(t):
    """strides (batch, head, row) of a [B, L, H, D] view with contiguous D"""
    assert t.stride(3) == 1
    return t.stride(0), t.stride(2), t.stride(1)


def keep_bits_ok(q, p_drop):
    """the flash forward writes (and the flash backward reads) a dropout keep bitmap for this
    attention: dropout on, bf16 head_dim 256 flash path"""
    return p_drop > 0 and q.shape[-1] == 256 and flash_bwd_eligible(q)


def keep_words(B, H, Lq, Lk):
    """int32 words of one launch's keep bitmap (s2h_attn_keep_words)"""
    return B * H * Lq * 2 * ((Lk + 63) // 64)


def attn_fwd(q, k, v, o, lse, scale, p_drop=0.0, seed=0, idx0=0, keep=None):
    """q [B, Lq, H, D], k/v [B, Lk, H, D] (any strides, D contiguous) -> o [B, Lq, H, D], lse [B, H, Lq] f32;
    keep: optional int32 [keep_words(...)] receiving the dropout keep bitmap (keep_bits_ok)"""
    _dev(q, k, v, o, lse)
    B, Lq, H, D = q.shape
    Lk = k.shape[1]
    nws = lib().s2h_attn_fwd_ws_bytes(dt(q), B, H, Lq, Lk, D)
    ws = torch.empty(nws, device=q.device, dtype=torch.uint8) if nws > 0 else None
    call("s2h_attn_fwd", dt(q), B, H, Lq, Lk, D, ptr(q), *_bhl(q), ptr(k), *_bhl(k), ptr(v), *_bhl(v),
         ptr(o), *_bhl(o), ptr(lse), float(scale), float(p_drop), int(seed) & (2**64 - 1), int(idx0),
         _keep_ptr(keep, B, H, Lq, Lk), ptr(ws), int(nws), stream())
    return o, lse


VFOLD_DV, VFOLD_COLS = 64, 72  # memory channels; columns of u' = [D M | rowsum(D) | 0 x 7]


def vfold_ok(q, mem):
    """the folded cross-attention's domain: bf16, one head of dim 256 (q [B, Lq, 1, 256]), 64-channel
    memory, flash-eligible query count"""
    return (q.dtype == torch.bfloat16 and q.shape[-1] == 256 and q.shape[-2] == 1 and mem.shape[-1] == VFOLD_DV
            and bool(lib().s2h_flash_bwd_ok(BF16, q.shape[1], 256)))


def _brs(t):
    """(batch, row) strides of a [B, L, (1,) C] view with contiguous channels"""
    assert t.stride(-1) == 1
    return t.stride(0), t.stride(1)


def attn_fwd_vfold(q, k, mem, u, lse, scale, p_drop=0.0, seed=0, idx0=0, keep=None):
    """q [B, Lq, 1, 256], k [B, Lk, 1, 256], mem [B, Lk, 1, 64] -> u [B, Lq, 1, 72] (u' = [D mem |
    rowsum(D) | 0]), lse [B, 1, Lq] (s2h_attn_fwd_vfold); keep as attn_fwd"""
    _dev(q, k, mem, u, lse)
    B, Lq = q.shape[0], q.shape[1]
    Lk = k.shape[1]
    nws = lib().s2h_attn_fwd_vfold_ws_bytes(B, Lq, Lk)
    ws = torch.empty(nws, device=q.device, dtype=torch.uint8) if nws > 0 else None
    call("s2h_attn_fwd_vfold", B, Lq, Lk, ptr(q), *_brs(q), ptr(k), *_brs(k), ptr(mem), *_brs(mem), ptr(u),
         *_brs(u), ptr(lse), float(scale), float(p_drop), int(seed) & (2**64 - 1), int(idx0),
         _keep_ptr(keep, B, 1, Lq, Lk), ptr(ws), int(nws), stream())
    return u, lse


def _rope_table_args(nfr, rope):
    """(cos, sin, period) checks and the per-frame row-count arrays of a fused inverse RoPE"""
    import ctypes
    cos, sin, period = rope[:3]
    _dev(cos, sin)
    assert cos.dtype == sin.dtype == torch.float32 and cos.is_contiguous() and sin.is_contiguous()

    def arr(n):  # (address, the ctypes array that must outlive the call)
        if n is None:
            return None
        assert len(n) == nfr
        a = (ctypes.c_int * nfr)(*[int(x) for x in n])
        return ctypes.addressof(a), a
    return ptr(cos), ptr(sin), int(period), arr


def flash_bwd_frames_vfold(nfr, bpf, lk, krow, idx0, q, k, mem, u, du, lse, dq, dk, scale, p_drop, seed, keep=None,
                           koff=None, rope=None, rope_q=None):
    """Frame-batched backward of attn_fwd_vfold (s2h_flash_bwd_frames_vfold): q / u / du / dq
    [nfr*bpf, Lq, 1, C] views, k / mem / dk PACKED [rows, 1, C] (frame f: bpf blocks of lk[f] rows
    from row krow[f]); keep / koff as flash_bwd_frames.  rope = (cos, sin, period, nrot per frame or
    None): dk comes out rotated back (the k projection's RoPE transposed, fused into the dK store);
    rope_q = query rows rotated per frame (same tables): dq rotated back in the dQ store
    (s2h_flash_bwd_frames_vfold_rope_qk)"""
    import ctypes
    _dev(q, k, mem, u, du, lse, dq, dk)
    B, Lq = q.shape[0], q.shape[1]
    assert B == nfr * bpf and len(lk) == nfr == len(krow) == len(idx0)
    di = torch.empty(B * Lq, device=q.device, dtype=torch.float32)
    alk = (ctypes.c_int * nfr)(*[int(x) for x in lk])
    akr = (ctypes.c_int64 * nfr)(*[int(x) for x in krow])
    aix = (ctypes.c_uint64 * nfr)(*[int(x) & (2**64 - 1) for x in idx0])
    kp = ako = None
    if keep is not None:
        assert keep.dtype == torch.int32 and len(koff) == nfr
        assert all(int(koff[f]) + keep_words(bpf, 1, Lq, lk[f]) <= keep.numel() for f in range(nfr))
        ako = (ctypes.c_int64 * nfr)(*[int(x) for x in koff])
        kp = ptr(keep)

    def rs(t):  # row stride of a packed [rows, 1, C] view
        assert t.stride(-1) == 1
        return t.stride(0)
    args = [nfr, bpf, Lq, ctypes.cast(alk, ctypes.c_void_p).value, ctypes.cast(akr, ctypes.c_void_p).value,
            ctypes.cast(aix, ctypes.c_void_p).value, ptr(q), *_brs(q), ptr(k), rs(k), ptr(mem), rs(mem), ptr(u), *_brs(u),
            ptr(du), *_brs(du), ptr(dq), *_brs(dq), ptr(dk), rs(dk), ptr(lse), ptr(di), float(scale), float(p_drop),
            int(seed) & (2**64 - 1), kp, ctypes.cast(ako, ctypes.c_void_p).value if kp is not None else None]
    if rope is None:
        assert rope_q is None
        call("s2h_flash_bwd_frames_vfold", *args, stream())
    else:
        pc, ps, period, arr = _rope_table_args(nfr, rope)
        ank, anq = arr(rope[3]), arr(rope_q)  # (pointer, keep-alive list)
        call("s2h_flash_bwd_frames_vfold_rope_qk", *args, pc, ps, period, ank[0] if ank else None,
             anq[0] if anq else None, stream())
    return dq, dk


def vfold_weight(wv, bv, out=None):
    """[Wv | bv | 0] bf16 [N, 72] from the bf16 weight [N, 64] and the fp32 bias [N]"""
    N, K = wv.shape
    if out is None:
        out = torch.empty(N, VFOLD_COLS, device=wv.device, dtype=torch.bfloat16)
    assert wv.dtype == torch.bfloat16 and wv.is_contiguous() and bv.dtype == torch.float32 and out.is_contiguous()
    call("s2h_vfold_weight", N, K, out.shape[1], ptr(wv), ptr(bv), ptr(out), stream())
    return out


def vfold_grad(g, gwv, gbv):
    """gwv [N, K] += g[:, :K], gbv [N] += g[:, K] (g fp32 [N, ld])"""
    N, ld = g.shape
    K = gwv.shape[1] if gwv is not None else VFOLD_DV
    call("s2h_vfold_grad", N, K, ld, ptr(g), ptr(gwv), ptr(gbv), stream())


def _keep_ptr(keep, B, H, Lq, Lk):
    if keep is None:
        return None
    assert keep.dtype == torch.int32 and keep.is_contiguous() and keep.numel() >= keep_words(B, H, Lq, Lk)
    return ptr(keep)


def attn_bwd(q, k, v, o, do, lse, dq, dk, dv, scale, p_drop=0.0, seed=0, idx0=0, keep=None):
    _dev(q, k, v, o, do, lse, dq, dk, dv)
    B, Lq, H, D = q.shape
    Lk = k.shape[1]
    di = torch.empty(B * H * Lq, device=q.device, dtype=torch.float32)
    nws = lib().s2h_attn_bwd_ws_bytes(dt(q), B, H, Lq, Lk, D)
    ws = torch.empty(nws, device=q.device, dtype=torch.uint8) if nws > 0 else None
    call("s2h_attn_bwd", dt(q), B, H, Lq, Lk, D,
         ptr(q), *_bhl(q), ptr(k), *_bhl(k), ptr(v), *_bhl(v), ptr(o), *_bhl(o), ptr(do), *_bhl(do),
         ptr(dq), *_bhl(dq), ptr(dk), *_bhl(dk), ptr(dv), *_bhl(dv),
         ptr(lse), ptr(di), float(scale), float(p_drop), int(seed) & (2**64 - 1), int(idx0),
         _keep_ptr(keep, B, H, Lq, Lk), ptr(ws), int(nws), stream())
    return dq, dk, dv


def flash_bwd_eligible(q):
    """the frame-batched flash backward's domain (bf16, head_dim 32..128 / 256, >= 128 query rows,
    flash path enabled): q [B, Lq, H, D]"""
    return bool(lib().s2h_flash_bwd_ok(dt(q), q.shape[1], q.shape[-1]))


def flash_bwd_frames(nfr, bpf, lk, krow, idx0, q, k, v, o, do, lse, dq, dk, dv, scale, p_drop, seed, keep=None,
                     koff=None, rope=None):
    """Frame-batched flash backward (s2h_flash_bwd_frames): q/o/do/dq [nfr*bpf, Lq, H, D] views,
    k/v/dk/dv PACKED [rows, H, D] views (frame f: bpf blocks of lk[f] rows from row krow[f]),
    lse [nfr*bpf, H, Lq]; frame f's dropout indices start at idx0[f]; keep (optional int32) holds
    frame f's forward keep bitmap from word koff[f].  rope = (cos, sin, period, query rows per frame):
    dq comes out rotated back (s2h_flash_bwd_frames_rope, the q projection's RoPE transposed in the
    dQ store; head dim 256)"""
    import ctypes
    _dev(q, k, v, o, do, lse, dq, dk, dv)
    B, Lq, H, D = q.shape
    assert B == nfr * bpf and len(lk) == nfr == len(krow) == len(idx0)
    di = torch.empty(B * H * Lq, device=q.device, dtype=torch.float32)
    alk = (ctypes.c_int * nfr)(*[int(x) for x in lk])
    akr = (ctypes.c_int64 * nfr)(*[int(x) for x in krow])
    aix = (ctypes.c_uint64 * nfr)(*[int(x) & (2**64 - 1) for x in idx0])
    kp = None
    if keep is not None:
        assert keep.dtype == torch.int32 and len(koff) == nfr
        assert all(int(koff[f]) + keep_words(bpf, H, Lq, lk[f]) <= keep.numel() for f in range(nfr))
        ako = (ctypes.c_int64 * nfr)(*[int(x) for x in koff])
        kp = ptr(keep)

    def hl(t):  # (head, row) strides of a packed [rows, H, D] view
        assert t.stride(-1) == 1
        return t.stride(1), t.stride(0)
    args = [nfr, bpf, H, Lq, D, ctypes.cast(alk, ctypes.c_void_p).value, ctypes.cast(akr, ctypes.c_void_p).value,
            ctypes.cast(aix, ctypes.c_void_p).value, ptr(q), *_bhl(q), ptr(k), *hl(k), ptr(v), *hl(v), ptr(o),
            *_bhl(o), ptr(do), *_bhl(do), ptr(dq), *_bhl(dq), ptr(dk), *hl(dk), ptr(dv), *hl(dv), ptr(lse), ptr(di),
            float(scale), float(p_drop), int(seed) & (2**64 - 1), kp,
            ctypes.cast(ako, ctypes.c_void_p).value if kp is not None else None]
    if rope is None:
        call("s2h_flash_bwd_frames", *args, stream())
    else:
        pc, ps, period, arr = _rope_table_args(nfr, rope)
        anq = arr(rope[3])
        call("s2h_flash_bwd_frames_rope", *args, pc, ps, period, anq[0], stream())
    return dq, dk, dv


# ------------------------------------------------------------ layernorm
def layernorm_fwd(x, gamma, beta, eps, y=None, add=None, add_bcast=False, xsum=None):
    """y = LN(x [+ add]) over the last dim; returns (y, mean, rstd).  If add is given the
    sum is written to xsum (residual stream)."""
    rows, C = _rows(x)
    if y is None:
        y = torch.empty(x.shape, device=x.device, dtype=x.dtype)
    mean = torch.empty(rows, device=x.device, dtype=torch.float32)
    rstd = torch.empty(rows, device=x.device, dtype=torch.float32)
    call("s2h_layernorm_fwd", dt(x), rows, C, ptr(x), x.stride(-2) if x.dim() > 1 else C,
         ptr(add), (add.stride(-2) if (add is not None and add.dim() > 1) else C), int(add_bcast), ptr(xsum),
         ptr(gamma), ptr(beta), float(eps), ptr(y), C, ptr(mean), ptr(rstd), stream())
    return y, mean, rstd


def layernorm_bwd(x, dy, gamma, mean, rstd, dx=None, accumulate=False, dgamma=None, dbeta=None, dres=None):
    """dx = LN'(dy) (+ dx when accumulate, or + dres); dgamma/dbeta += weight gradients."""
    rows, C = _rows(x)
    if dx is None:
        dx = torch.empty(x.shape, device=x.device, dtype=x.dtype)
    if dres is not None:
        assert dres.is_contiguous() and dres.dtype == x.dtype and dres.numel() == x.numel() and not accumulate
    ws = None
    if dgamma is not None:  # (unused when the library defers the gamma / beta sums)
        nbytes = lib().s2h_layernorm_bwd_ws_bytes(dt(x), rows, C)
        ws = torch.empty(max(nbytes // 4, 1), device=x.device, dtype=torch.float32)
    call("s2h_layernorm_bwd", dt(x), rows, C, ptr(x), C, ptr(dy), C, ptr(gamma), ptr(mean), ptr(rstd),
         ptr(dx), C, int(accumulate), ptr(dres), C, ptr(dgamma), ptr(dbeta), ptr(ws), stream())
    return dx


# ----------------------------------------------------------- elementwise
def add(a, b, out=None, alpha=1.0, beta=1.0):
    ref = a if a is not None else b
    if out is None:
        out = torch.empty_like(ref)
    call("s2h_add", dt(ref), ref.numel(), ptr(a), ptr(b), float(alpha), float(beta), ptr(out), stream())
    return out


def add_bcast(a, b, out=None, alpha=1.0, beta=1.0, b_period=1, shape=None):
    """out[i, :] = alpha*a[i, :] + beta*b[i % b_period, :]  (a may be None -> broadcast copy)"""
    inner = b.numel() // b_period
    if out is None:
        out = torch.empty(shape if shape is not None else a.shape, device=b.device, dtype=b.dtype)
    outer = out.numel() // inner
    call("s2h_add_bcast", dt(out), outer, inner, ptr(a), float(alpha), ptr(b), b_period, float(beta), ptr(out),
         stream())
    return out


def act_fwd(x, act, out=None, scale=1.0, shift=0.0):
    if out is None:
        out = torch.empty_like(x)
    call("s2h_act_fwd", dt(x), x.numel(), ptr(x), ACT[act], float(scale), float(shift), ptr(out), stream())
    return out


def act_dropout_bwd(x_pre, dy, act, p, seed, dx=None, idx0=0):
    """dx = act'(x_pre) * dropout_mask(seed) / (1 - p) * dy (one pass; x_pre None = no act)"""
    if dx is None:
        dx = torch.empty_like(dy)
    call("s2h_act_dropout_bwd", dt(dy), dy.numel(), ptr(x_pre), ptr(dy), ACT[act], float(p), int(seed) & (2**64 - 1),
         int(idx0), ptr(dx), stream())
    return dx


def relu_mask_bwd(y, dy, scale=1.0, dx=None):
    """dx = scale * [y > 0] * dy -- ReLU (-> dropout) backward from the layer output y"""
    assert y.is_contiguous() and dy.is_contiguous() and y.numel() == dy.numel() and y.dtype == dy.dtype
    if dx is None:
        dx = torch.empty_like(dy)
    call("s2h_relu_mask_bwd", dt(dy), dy.numel(), ptr(y), ptr(dy), float(scale), ptr(dx), stream())
    return dx


def act_bwd(x_pre, dy, act, dx=None, accumulate=False):
    if dx is None:
        dx = torch.empty_like(dy)
    call("s2h_act_bwd", dt(dy), dy.numel(), ptr(x_pre), ptr(dy), ACT[act], ptr(dx), int(accumulate), stream())
    return dx


def cast(x, dtype, out=None):
    if out is None:
        out = torch.empty(x.shape, device=x.device, dtype=dtype)
    call("s2h_cast", dt(x), dt(out), x.numel(), ptr(x), ptr(out), stream())
    return out


def dropout(b, p, seed, a=None, out=None, idx0=0):
    """out = (a +) keep*b/(1-p) with the counter-hash mask of (seed, flat index)"""
    if out is None:
        out = torch.empty_like(b)
    call("s2h_dropout", dt(b), b.numel(), ptr(a), ptr(b), float(p), int(seed) & (2**64 - 1), int(idx0), ptr(out),
         stream())
    return out


def rope(x, y, nrot, cos, sin, period, inverse=False):
    """x/y [Bt, L, D] views (D contiguous): rotate pairs of the first nrot rows of every batch."""
    Bt, L, D = x.shape
    call("s2h_rope", dt(x), Bt, nrot, D, ptr(x), x.stride(0), x.stride(1), ptr(y), y.stride(0), y.stride(1),
         ptr(cos), ptr(sin), period, int(inverse), stream())
    return y


def maxpool2(x, out=None):
    """x [B, H, W, C] (pixel stride x.stride(2), C contiguous) -> [B, H/2, W/2, C]"""
    B, H, W, C = x.shape
    assert x.stride(1) == W * x.stride(2) and x.stride(0) == H * x.stride(1) and x.stride(3) == 1
    if out is None:
        out = torch.empty(B, H // 2, W // 2, C, device=x.device, dtype=x.dtype)
    call("s2h_maxpool2_fwd", dt(x), B, H, W, C, ptr(x), x.stride(2), ptr(out), stream())
    return out


def maxpool2_bwd(x, dy, dx):
    B, H, W, C = x.shape
    call("s2h_maxpool2_bwd", dt(x), B, H, W, C, ptr(x), x.stride(2), ptr(dy), ptr(dx), dx.stride(2), stream())
    return dx


def window_partition(x, ws, out=None, accumulate=False):
    B, H, W, C = x.shape
    nh, nw = -(-H // ws), -(-W // ws)
    if out is None:
        out = torch.empty(B * nh * nw, ws, ws, C, device=x.device, dtype=x.dtype)
    call("s2h_window", dt(x), B, H, W, C, ws, ptr(x), ptr(out), 0, int(accumulate), stream())
    return out


def window_pad(x, ws, padrow, out=None):
    """window_partition of a projection's output x [B, H, W, C] with the padded positions = padrow
    (fp32 [C], the projection's bias): [B * nh * nw, ws, ws, C]"""
    B, H, W, C = x.shape
    nh, nw = -(-H // ws), -(-W // ws)
    assert padrow.dtype == torch.float32 and padrow.numel() == C and padrow.is_contiguous() and x.is_contiguous()
    if out is None:
        out = torch.empty(B * nh * nw, ws, ws, C, device=x.device, dtype=x.dtype)
    _dev(x, padrow, out)
    call("s2h_window_pad", dt(x), B, H, W, C, ws, ptr(x), ptr(padrow), ptr(out), stream())
    return out


def window_pad_colsum(win, ws, B, H, W, out):
    """out (fp32 [C]) += the column sums of win's padded rows (window_pad's bias gradient)"""
    C = win.shape[-1]
    assert out.dtype == torch.float32 and out.numel() == C and out.is_contiguous() and win.is_contiguous()
    _dev(win, out)
    call("s2h_window_pad_colsum", dt(win), B, H, W, C, ws, ptr(win), ptr(out), stream())
    return out


def window_unpartition(win, ws, B, H, W, out=None, accumulate=False):
    C = win.shape[-1]
    if out is None:
        out = torch.empty(B, H, W, C, device=win.device, dtype=win.dtype)
    call("s2h_window", dt(win), B, H, W, C, ws, ptr(win), ptr(out), 1, int(accumulate), stream())
    return out


# S2H_COPY_BATCH=0: one Tensor.copy_ per pair (A/B of s2h_copy2d_batch)
_COPY_BATCH = os.environ.get("S2H_COPY_BATCH", "1") != "0"


def _pair_rows(src, dst):
    """(rows, row_bytes, src_pitch, dst_pitch) of the copy dst <- src (same shape and dtype) as a
    2-D byte copy, or None when the layouts do not reduce to one (contiguous rows, uniform pitch)"""
    if src.shape != dst.shape or src.dtype != dst.dtype:
        return None
    dims = [d for d in range(src.dim()) if src.shape[d] != 1]
    es = src.element_size()
    inner, k = 1, len(dims)
    while k > 0 and src.stride(dims[k - 1]) == inner and dst.stride(dims[k - 1]) == inner:
        inner *= src.shape[dims[k - 1]]
        k -= 1
    lead = dims[:k]
    if not lead:
        return 1, inner * es, inner * es, inner * es
    rows = 1
    for a, b in zip(lead[:-1], lead[1:]):  # the leading dims must collapse into one pitch
        if src.stride(a) != src.stride(b) * src.shape[b] or dst.stride(a) != dst.stride(b) * dst.shape[b]:
            return None
    for d in lead:
        rows *= src.shape[d]
    return rows, inner * es, src.stride(lead[-1]) * es, dst.stride(lead[-1]) * es


def copy_segments(pairs):
    """dst.copy_(src) for every (src, dst) pair, up to 16 pairs per launch (s2h_copy2d_batch): the
    memory bank assembly of a tracked frame (sam2_base.py:649-676) and the tracking loop's gradient
    packing.  A pair whose layout is not a 4-B aligned 2-D copy goes through Tensor.copy_ (16-B
    aligned pairs move in 16-B pieces, the rest in 4-B pieces)."""
    import ctypes
    if not _COPY_BATCH:
        for src, dst in pairs:
            dst.copy_(src)
        return
    segs = []
    for src, dst in pairs:
        r = _pair_rows(src, dst) if src.is_cuda and dst.is_cuda else None
        if r is None or src.numel() == 0 or any(v % 4 for v in r[1:]) or src.data_ptr() % 4 or dst.data_ptr() % 4 \
                or (r[0] > 1 and r[3] < r[1]):  # overlapping destination rows (a source pitch of 0 broadcasts)
            dst.copy_(src)
            continue
        segs.append((src.data_ptr(), dst.data_ptr()) + r)
    for i in range(0, len(segs), 16):
        chunk = segs[i:i + 16]
        n = len(chunk)
        P, L = ctypes.c_void_p * n, ctypes.c_int64 * n
        arrs = [P(*[c[0] for c in chunk]), P(*[c[1] for c in chunk])] + [L(*[c[j] for c in chunk]) for j in range(2, 6)]
        call("s2h_copy2d_batch", n, *arrs, stream())


def up2_add(lat, prev, out=None):
    B, H, W, C = lat.shape
    if out is None:
        out = torch.empty_like(lat)
    call("s2h_up2_add", dt(lat), B, H, W, C, ptr(lat), ptr(prev), ptr(out), stream())
    return out


def pool2_sum(dout, dprev, accumulate=False):
    B, Ho, Wo, C = dprev.shape
    call("s2h_pool2_sum", dt(dout), B, Ho, Wo, C, ptr(dout), ptr(dprev), int(accumulate), stream())
    return dprev


def bilinear(x, ho, wo, out=None):
    """x [N, hi, wi] f32 -> [N, ho, wo] (align_corners=False)"""
    N, hi, wi = x.shape
    if out is None:
        out = torch.empty(N, ho, wo, device=x.device, dtype=torch.float32)
    call("s2h_bilinear_fwd", N, hi, wi, ho, wo, ptr(x), ptr(out), stream())
    return out


def bilinear_bwd(dy, hi, wi, dx=None):
    N, ho, wo = dy.shape
    if dx is None:
        dx = torch.empty(N, hi, wi, device=dy.device, dtype=torch.float32)
    call("s2h_bilinear_bwd", N, hi, wi, ho, wo, ptr(dy), ptr(dx), stream())
    return dx


def colsum(x, out, accumulate=True):
    """out (fp32 [C]) (+)= x.reshape(-1, C).sum(0)"""
    rows, C = _rows(x)
    call("s2h_colsum", dt(x), rows, C, ptr(x), x.stride(-2) if x.dim() > 1 else C, ptr(out), int(accumulate),
         stream())
    return out


def colsum_seg(x, rows, offs, dsts, out):
    """out[dsts[s]] += x[offs[s]:offs[s] + rows].sum(0) for every segment s (x [R, C] row-contiguous,
    out fp32 [*, C]); one launch for up to 64 segments"""
    import ctypes
    C = x.shape[-1]
    _dev(x, out)
    assert x.stride(-1) == 1 and out.dtype == torch.float32 and out.is_contiguous() and len(offs) == len(dsts) <= 64
    o = (ctypes.c_int64 * len(offs))(*[int(v) for v in offs])
    d = (ctypes.c_int * len(dsts))(*[int(v) for v in dsts])
    call("s2h_colsum_seg", dt(x), len(offs), int(rows), C, ptr(x), x.stride(-2), ctypes.addressof(o),
         ctypes.addressof(d), ptr(out), stream())
    return out


def memory_pos(pos, tpos, idx, out):
    """out[j * L + l] = pos[l] + tpos[idx[j]] for j < len(idx) <= 16 (pos [L, C], tpos [*, C], out [n L, C],
    all contiguous, one dtype)"""
    import ctypes
    L, C = pos.shape
    _dev(pos, tpos, out)
    assert pos.is_contiguous() and tpos.is_contiguous() and out.is_contiguous() and len(idx) <= 16
    assert pos.dtype == tpos.dtype == out.dtype and out.numel() == len(idx) * L * C
    ix = (ctypes.c_int * len(idx))(*[int(v) for v in idx])
    call("s2h_memory_pos", dt(out), len(idx), L, C, ptr(pos), ptr(tpos), ctypes.addressof(ix), ptr(out), stream())
    return out


def sum_outer(x, out, accumulate=False):
    """out[j] = sum_o x[o, j]  (same dtype as x)"""
    O = x.shape[0]
    call("s2h_sum_outer", dt(x), O, x.numel() // O, ptr(x), ptr(out), int(accumulate), stream())
    return out


def sum_outer_batched(x3, out, accumulate=False):
    """out[f] (+)= x3[f].sum(0) for x3 [F, O, inner] (one launch; the values of F sum_outer calls)"""
    F, O, inner = x3.shape
    assert x3.is_contiguous() and out.is_contiguous() and out.numel() == F * inner and out.dtype == x3.dtype
    call("s2h_sum_outer_batched", dt(x3), F, O, inner, ptr(x3), ptr(out), int(accumulate), stream())
    return out


def im2col(x, kh, kw, stride, pad, pad8=False):
    """[B*Ho*Wo, C*kh*kw] patches; pad8: a view of rows padded to a multiple of 8 elements (zeros), so
    the GEMMs reading it (the patch embedding's 147 columns) get 16-B aligned rows"""
    B, H, W, C = x.shape
    Ho = (H + 2 * pad - kh) // stride + 1
    Wo = (W + 2 * pad - kw) // stride + 1
    Kc = C * kh * kw
    ld = (Kc + 7) // 8 * 8 if pad8 else Kc
    buf = torch.empty(B * Ho * Wo, ld, device=x.device, dtype=x.dtype)
    call("s2h_im2col", dt(x), B, H, W, C, kh, kw, stride, pad, Ho, Wo, ld, ptr(x), ptr(buf), stream())
    return (buf[:, :Kc] if ld != Kc else buf), Ho, Wo


def dwconv(x, w, bias, pad):
    B, H, W, C = x.shape
    K = w.shape[-1]
    out = torch.empty_like(x)
    call("s2h_dwconv", dt(x), B, H, W, C, K, pad, ptr(x), ptr(w), ptr(bias), ptr(out), stream())
    return out


def convt2_scatter(Y, B, H, W, Co, bias=None, add=None, out=None):
    if out is None:
        out = torch.empty(B, 2 * H, 2 * W, Co, device=Y.device, dtype=Y.dtype)
    call("s2h_convt2", dt(Y), B, H, W, Co, ptr(Y), ptr(bias), ptr(add), ptr(out), 0, stream())
    return out


# S2H_CONVT_DIRECT=0: the scalar scatter + a separate (broadcast) add (A/B)
_CONVT_DIRECT = os.environ.get("S2H_CONVT_DIRECT", "1") == "1"


def convt2_direct():
    return _CONVT_DIRECT


def convt2_store(Y, B, H, W, Co, bias=None, add=None, out=None):
    """out = scatter(Y) + bias (+ add: [B or 1, 2H, 2W, Co], broadcast over B when it has one batch),
    vectorised, one rounding (s2h_convt2_store)"""
    if out is None:
        out = torch.empty(B, 2 * H, 2 * W, Co, device=Y.device, dtype=Y.dtype)
    bc = 0
    if add is not None:
        assert add.is_contiguous() and add.dtype == Y.dtype and add.shape[1:] == out.shape[1:]
        assert add.shape[0] in (1, B)
        bc = int(add.shape[0] == 1 and B > 1)
    call("s2h_convt2_store", dt(Y), B, H, W, Co, ptr(Y), ptr(bias), ptr(add), bc, ptr(out), stream())
    return out


def convt2_tail(Y, B, H, W, Co, bias, add, hyper, pre, post, masks):
    """pre = convt2_store(Y) + bias + add, post = gelu(pre), masks[b] = post[b] . hyper[b] (s2h_convt2_tail)"""
    bc = 0
    if add is not None:
        assert add.is_contiguous() and add.dtype == Y.dtype and add.shape[0] in (1, B)
        bc = int(add.shape[0] == 1 and B > 1)
    assert hyper.is_contiguous() and hyper.numel() == B * Co and pre.is_contiguous() and post.is_contiguous()
    call("s2h_convt2_tail", dt(Y), B, H, W, Co, ptr(Y), ptr(bias), ptr(add), bc, ptr(hyper), ptr(pre), ptr(post),
         ptr(masks), stream())
    return masks


def convt2_tail_enabled():
    return os.environ.get("S2H_CONVT_TAIL", "1") == "1"


def convt2_gather(dout, B, H, W, Co, dY=None):
    if dY is None:
        dY = torch.empty(B * H * W, 4 * Co, device=dout.device, dtype=dout.dtype)
    call("s2h_convt2", dt(dout), B, H, W, Co, ptr(dout), None, None, ptr(dY), 1, stream())
    return dY


def row_gate(x, gate, fill, out=None, backward=False):
    rows = x.shape[0]
    if out is None:
        out = torch.empty_like(x)
    call("s2h_row_gate", dt(x), rows, x.numel() // rows, ptr(x), ptr(gate), float(fill), ptr(out), int(backward),
         stream())
    return out


def row_gate_cast(x, gate, fill, dtype, out=None, backward=False, gate_out=None):
    """row_gate with the output in `dtype` (s2h_row_gate_cast); gate_out: the gate copied beside it"""
    rows = x.shape[0]
    if out is None:
        out = torch.empty(x.shape, device=x.device, dtype=dtype)
    call("s2h_row_gate_cast", dt(x), dt(out), rows, x.numel() // rows, ptr(x), ptr(gate), float(fill), ptr(out),
         int(backward), ptr(gate_out), stream())
    return out


def gate_mix(x, gate, vec, scale_x=False, out=None):
    rows = x.shape[0]
    if out is None:
        out = torch.empty_like(x)
    call("s2h_gate_mix", dt(x), rows, x.numel() // rows, ptr(x), ptr(gate), ptr(vec), vec.numel(), int(scale_x),
         ptr(out), stream())
    return out


# ------------------------------------------------------------------ loss
NSTAT = 6


def mask_stats(x, tgt, inv_temp=1.0, stats=None):
    """x [N, P] f32 logits, tgt [N, P] uint8/bool (or None) -> stats [N, 6] f32"""
    N, P = x.shape
    if stats is None:
        stats = torch.empty(N, NSTAT, device=x.device, dtype=torch.float32)
    call("s2h_mask_stats", N, P, ptr(x), x.stride(0), ptr(tgt), tgt.stride(0) if tgt is not None else 0,
         float(inv_temp), ptr(stats), stream())
    return stats


def mask_loss_finalize(stats, pred_iou, valid, P, weights, gscale, losses, coef):
    N = stats.shape[0]
    call("s2h_mask_loss_finalize", N, P, ptr(stats), ptr(pred_iou), ptr(valid), float(weights[0]),
         float(weights[1]), float(weights[2]), float(gscale), ptr(losses), ptr(coef), stream())


def mask_loss_bwd(x, tgt, coef, inv_temp, dx, gtot=None, dious=None):
    N, P = x.shape
    call("s2h_mask_loss_bwd", N, P, ptr(x), x.stride(0), ptr(tgt), tgt.stride(0), float(inv_temp), ptr(coef),
         ptr(dx), dx.stride(0), ptr(gtot), ptr(dious), stream())
    return dx


def bce_stats(x, tgt, inv_temp=1.0, pos_weight=None):
    """x [N, P] f32 logits, tgt [N, P] uint8 -> stats [N, 2] (bce sum, target sum)"""
    N, P = x.shape
    stats = torch.empty(N, 2, device=x.device, dtype=torch.float32)
    call("s2h_bce_stats", N, P, ptr(x), x.stride(0), ptr(tgt), tgt.stride(0), float(inv_temp), ptr(pos_weight),
         ptr(stats), stream())
    return stats


def bce_finalize(stats, P, reduction, frame_scale, losses, coef):
    call("s2h_bce_finalize", stats.shape[0], P, ptr(stats), int(reduction), float(frame_scale), ptr(losses),
         ptr(coef), stream())


def bce_bwd(x, tgt, inv_temp, pos_weight, coef, dx, gtot=None):
    N, P = x.shape
    call("s2h_bce_bwd", N, P, ptr(x), x.stride(0), ptr(tgt), tgt.stride(0), float(inv_temp), ptr(pos_weight),
         ptr(coef), ptr(gtot), ptr(dx), dx.stride(0), stream())
    return dx


def group_max(x, cat_off, cat_obj, ncat, out, arg):
    P = x.shape[1]
    call("s2h_group_max_fwd", ncat, P, ptr(cat_off), ptr(cat_obj), ptr(x), x.stride(0), ptr(out), out.stride(0),
         ptr(arg), stream())
    return out


def group_max_bwd(dy, obj_cat, arg, dx):
    O, P = dx.shape
    call("s2h_group_max_bwd", O, P, ptr(obj_cat), ptr(arg), ptr(dy), dy.stride(0), ptr(dx), dx.stride(0), stream())
    return dx


def group_wavg(x, stats, cat_off, cat_obj, ncat, out):
    K = x.shape[1]
    call("s2h_group_wavg_fwd", ncat, K, ptr(cat_off), ptr(cat_obj), ptr(stats), ptr(x), ptr(out), stream())
    return out


def group_wavg_bwd(x, y, dy, stats, obj_cat, cat_off, dx, dw):
    O, K = x.shape
    call("s2h_group_wavg_bwd", O, K, ptr(obj_cat), ptr(cat_off), ptr(stats), ptr(x), ptr(y), ptr(dy), ptr(dx),
         ptr(dw), stream())


def sigmoid_grad_axpy(x, coef, dx):
    R, P = x.shape
    call("s2h_sigmoid_grad_axpy", R, P, ptr(x), x.stride(0), ptr(coef), ptr(dx), dx.stride(0), stream())
    return dx


# ------------------------------------------------------------- optimizer
def grad_norm(g, max_norm, ws, out, grad_scale=1.0):
    """out[0] = ||grad_scale*g||, out[1] = grad_scale * clip coefficient (device scalars)"""
    call("s2h_grad_norm", g.numel(), ptr(g), ptr(ws), float(max_norm), float(grad_scale), ptr(out), stream())
    return out


def adamw(p, g, m, v, clip, lr, beta1, beta2, eps, wd, step, shadow=None):
    call("s2h_adamw", p.numel(), ptr(p), ptr(g), ptr(m), ptr(v), ptr(clip), float(lr), float(beta1), float(beta2),
         float(eps), float(wd), int(step), ptr(shadow), stream())


def pos_embed(Y, win, h, w, out):
    """out [h, w, C] = Y [C, h, w] + tile(win [C, ws, ws])"""
    C = Y.shape[0]
    ws = win.shape[-1]
    call("s2h_pos_embed", dt(out), C, h, w, ws, ptr(Y), ptr(win.contiguous()), ptr(out), stream())
    return out


def pos_embed_bwd(dout, dY, dwin, ws):
    h, w, C = dout.shape
    call("s2h_pos_embed_bwd", dt(dout), C, h, w, ws, ptr(dout), ptr(dY), ptr(dwin), stream())


def point_embed(pe, labels, table, out, labels_out=None):
    R, D = pe.shape
    assert labels_out is None or (labels_out.dtype == torch.int32 and labels_out.numel() == R)
    call("s2h_point_embed", dt(out), R, D, ptr(pe), ptr(labels), ptr(table), ptr(out), ptr(labels_out), stream())
    return out


def point_embed_bwd(labels, dout, dtable):
    R, D = dout.shape
    call("s2h_point_embed_bwd", dt(dout), R, D, ptr(labels), ptr(dout), ptr(dtable), stream())


def point_embed_bwd_rows(labels, dout, rows):
    """point_embed_bwd into 5 separate fp32 [D] rows (each accumulated in row order)"""
    import ctypes
    R, D = dout.shape
    assert len(rows) == 5 and all(r.dtype == torch.float32 and r.numel() == D and r.is_contiguous() for r in rows)
    arr = (ctypes.c_void_p * 5)(*[ptr(r) for r in rows])
    call("s2h_point_embed_bwd_rows", dt(dout), R, D, ptr(labels), ptr(dout), ctypes.addressof(arr), stream())


def version():
    from ._lib import lib
    return lib().s2h_version()


_ = math


def mask_down_stage(x, w, bias, gamma, beta, eps, *, logits=None, scale=1.0, shift=0.0, dtype=None):
    """Fused MaskDownSampler stage: GELU(LN2d(conv3x3/2(x))) on NHWC x [O, H, W, cin];
    or, with `logits` ([O, H, W] fp32), on sigmoid(logits) * scale + shift (cin = 1)."""
    cout, cin = w.shape[0], w.shape[1]
    assert tuple(w.shape[2:]) == (3, 3) and w.dtype == torch.float32 and w.is_contiguous()
    src = logits if logits is not None else x
    assert src.is_contiguous()
    O, H, W = src.shape[0], src.shape[1], src.shape[2]
    if logits is not None:
        assert logits.dtype == torch.float32 and cin == 1 and dtype is not None
    else:
        assert x.shape[-1] == cin
        dtype = x.dtype
    y = torch.empty(O, (H + 1) // 2, (W + 1) // 2, cout, device=src.device, dtype=dtype)
    call("s2h_mask_down_stage", BF16 if dtype == torch.bfloat16 else F32, O, H, W, cin, cout, ptr(src),
         int(logits is not None), float(scale), float(shift), ptr(w), ptr(bias), ptr(gamma), ptr(beta), float(eps),
         ptr(y), stream())
    return y


def mask_eval_counts(logits, tgt):
    """[N, 4] int64 counts (|pred & gt|, |pred | gt|, |pred|, |gt|) per category, pred = logits > 0.
    logits [N, ...] fp32, tgt [N, ...] bool/uint8 of the same pixel count."""
    N = logits.shape[0]
    x = logits.reshape(N, -1)
    t = tgt.reshape(N, -1)
    if t.dtype == torch.bool:
        t = t.view(torch.uint8)
    assert x.dtype == torch.float32 and t.dtype == torch.uint8 and x.shape == t.shape
    assert x.stride(-1) == 1 and t.stride(-1) == 1
    out = torch.empty(N, 4, device=x.device, dtype=torch.int64)
    call("s2h_mask_eval_counts", N, x.shape[1], ptr(x), x.stride(0), ptr(t), t.stride(0), ptr(out), stream())
    return out
