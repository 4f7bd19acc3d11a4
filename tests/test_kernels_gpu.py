"""Per-kernel numerics of libsam2hip against plain PyTorch fp32 references of the
same op (run on the GPU box).  fp32 path (f32-input MFMA) must match to ~1e-5
relative; bf16 path within bf16 rounding of the inputs."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _ops():
    from sam2_video.kernels import ops
    return ops


def _cpu_conv(fn, x, w, b, **kw):
    """fp32 torch convolution evaluated on the host (the references never go through MIOpen's
    GPU solvers: its conv-transpose solver faulted on a fresh box), returned on x's device."""
    return fn(x.float().cpu(), w.float().cpu(), None if b is None else b.float().cpu(), **kw).to(x.device)


def _close(a, b, tol):
    a = a.float()
    b = b.float()
    err = (a - b).abs().max().item()
    scale = b.abs().max().item() + 1e-6
    assert err <= tol * scale, f"max err {err:.3e} vs scale {scale:.3e} (tol {tol})"


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-5), (torch.bfloat16, 1e-2)])
@pytest.mark.parametrize("M,N,K", [(1, 1, 1), (7, 13, 5), (64, 64, 32), (300, 257, 129), (1024, 768, 256),
                                   (4100, 130, 200)])
def test_linear_fwd_dgrad_wgrad(dtype, tol, M, N, K):
    ops = _ops()
    torch.manual_seed(0)
    x = torch.randn(M, K, device=DEV).to(dtype)
    w = torch.randn(N, K, device=DEV).to(dtype)
    b = torch.randn(N, device=DEV)
    y = ops.linear(x, w, b)
    ref = x.float() @ w.float().t() + b
    _close(y, ref, tol)
    for act in ("relu", "gelu"):
        pre = torch.empty(M, N, device=DEV, dtype=dtype)
        y = ops.linear(x, w, b, act=act, pre=pre)
        r = torch.relu(ref) if act == "relu" else torch.nn.functional.gelu(ref)
        _close(y, r, tol)
        _close(pre, ref, tol)
    dy = torch.randn(M, N, device=DEV).to(dtype)
    dx = ops.linear_dgrad(dy, w)
    _close(dx, dy.float() @ w.float(), tol)
    dw = torch.zeros(N, K, device=DEV)
    db = torch.zeros(N, device=DEV)
    ops.linear_wgrad(dy, x, dw, db=db)
    ops.linear_wgrad(dy, x, dw, db=db)  # accumulates
    _close(dw, 2 * dy.float().t() @ x.float(), tol)
    _close(db, 2 * dy.float().sum(0), 1e-4)
    ops.linear_wgrad(dy, x, dw, accumulate=False, db=db)
    _close(dw, dy.float().t() @ x.float(), tol)
    _close(db, dy.float().sum(0), 1e-4)
    r = torch.randn(M, N, device=DEV).to(dtype)
    y = ops.linear(x, w, b, residual=r)
    _close(y, ref + r.float(), tol)


@pytest.mark.parametrize("M,N,K", [(1024, 768, 256), (300, 264, 200), (4104, 136, 72), (64, 64, 64), (520, 2048, 1032),
                                   (13312, 256, 2048)])
@pytest.mark.parametrize("layout", ["nt", "nn", "tn", "tt"])
def test_gemm_lds_dma_path(M, N, K, layout):
    """LDS-DMA GEMM (swizzled images, K tail zeroing, XCD remap) vs torch, every operand layout,
    plus the fused epilogue (bias, GELU, residual) and fp32 split-K output."""
    ops = _ops()
    torch.manual_seed(7)
    bf = torch.bfloat16
    a = torch.randn(M, K, device=DEV).to(bf) if layout[0] == "n" else torch.randn(K, M, device=DEV).to(bf).t()
    b = torch.randn(K, N, device=DEV).to(bf) if layout[1] == "n" else torch.randn(N, K, device=DEV).to(bf).t()
    ref = a.float() @ b.float()
    kw = dict(M=M, N=N, K=K, lda_m=a.stride(0), lda_k=a.stride(1), ldb_k=b.stride(0), ldb_n=b.stride(1), ldc=N)
    out = torch.empty(M, N, device=DEV, dtype=bf)
    ops.gemm(a, b, out, **kw)
    _close(out, ref, 1e-2)
    bias = torch.randn(N, device=DEV)
    res = torch.randn(M, N, device=DEV).to(bf)
    ops.gemm(a, b, out, bias=bias, residual=res, ldr=N, act=2, **kw)
    _close(out, torch.nn.functional.gelu(ref + bias) + res.float(), 1e-2)
    o32 = torch.full((M, N), 3.0, device=DEV)
    ops.gemm(a, b, o32, beta=1.0, **kw)
    _close(o32, ref + 3.0, 2e-3)


@pytest.mark.parametrize("cfg", [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24,
                                 25, 26, 27, 28, 29, 30, -1])
@pytest.mark.parametrize("M,N,K", [(1000, 520, 200), (600, 264, 1100), (13312, 256, 256), (333, 136, 72)])
@pytest.mark.parametrize("layout", ["nt", "nn", "tn", "tt"])
def test_gemm_every_tiling(cfg, M, N, K, layout):
    """each forced tiling (64^2, 128^2 2/3-deep ring, 256x128, 256^2, 128x256, register-staged)
    on ragged shapes and every operand layout, with the fused epilogue and fp32 accumulate"""
    from sam2_video.kernels import _lib
    ops = _ops()
    torch.manual_seed(11)
    bf = torch.bfloat16
    a = torch.randn(M, K, device=DEV).to(bf) if layout[0] == "n" else torch.randn(K, M, device=DEV).to(bf).t()
    b = torch.randn(K, N, device=DEV).to(bf) if layout[1] == "n" else torch.randn(N, K, device=DEV).to(bf).t()
    ref = a.float() @ b.float()
    kw = dict(M=M, N=N, K=K, lda_m=a.stride(0), lda_k=a.stride(1), ldb_k=b.stride(0), ldb_n=b.stride(1), ldc=N)
    prev = _lib.lib().s2h_gemm_config(cfg)
    try:
        out = torch.empty(M, N, device=DEV, dtype=bf)
        bias = torch.randn(N, device=DEV)
        res = torch.randn(M, N, device=DEV).to(bf)
        ops.gemm(a, b, out, bias=bias, residual=res, ldr=N, act=1, **kw)
        _close(out, torch.relu(ref + bias) + res.float(), 1e-2)
        o32 = torch.full((M, N), 3.0, device=DEV)
        ops.gemm(a, b, o32, beta=1.0, **kw)
        _close(o32, ref + 3.0, 2e-3)
    finally:
        _lib.lib().s2h_gemm_config(prev)


@pytest.mark.parametrize("pcfg,cfg", [(20, 1), (21, 7), (22, 11), (23, 18), (24, 13)])
@pytest.mark.parametrize("batch,M,N,K", [(3, 1000, 520, 200), (2, 13312, 256, 256), (1, 64, 64, 64), (5, 70, 24, 40)])
def test_gemm_wave_grid_4x1_matches_2x2(pcfg, cfg, batch, M, N, K):
    """the 4 x 1 wave grids (every wave owns whole 64-column tile rows: full-line epilogue stores)
    are bit-identical to the 2 x 2 grids of the same tile and ring -- same K order per 16x16
    accumulator, same epilogue incl. the dropout hash of each output index -- on batched, ragged
    and single-tile problems"""
    from sam2_video.kernels import _lib
    ops = _ops()
    torch.manual_seed(5)
    bf = torch.bfloat16
    a = torch.randn(batch, M, K, device=DEV).to(bf)
    b = torch.randn(batch, N, K, device=DEV).to(bf)
    bias = torch.randn(N, device=DEV)
    res = torch.randn(batch, M, N, device=DEV).to(bf)
    ref = torch.relu(a.float() @ b.float().transpose(1, 2) + bias) + res.float()
    for drop in (0.1, 0.0):
        kw = dict(M=M, N=N, K=K, lda_m=K, lda_k=1, ldb_k=1, ldb_n=K, ldc=N, batch=batch, sA=M * K, sB=N * K,
                  sC=M * N, bias=bias, residual=res, ldr=N, sR=M * N, act=1, drop_p=drop, seed=77)
        outs = []
        for c in (pcfg, cfg):
            prev = _lib.lib().s2h_gemm_config(c)
            try:
                out = torch.full((batch, M, N), float("nan"), device=DEV, dtype=bf)
                ops.gemm(a, b, out, **kw)
                outs.append(out)
            finally:
                _lib.lib().s2h_gemm_config(prev)
        torch.cuda.synchronize()
        assert not torch.isnan(outs[0].float()).any()
        assert torch.equal(outs[0], outs[1])
    _close(outs[0], ref, 1e-2)


@pytest.mark.parametrize("rows,N,K", [(20000, 336, 112), (131072, 112, 336), (13312, 256, 256), (4099, 130, 77)])
def test_wgrad_split_k(rows, N, K):
    """Weight gradients reduce over 10^4-10^5 rows into few output tiles: the bf16 GEMM
    splits the reduction over workgroups with fp32 atomics (accumulate semantics)."""
    ops = _ops()
    torch.manual_seed(1)
    dy = torch.randn(rows, N, device=DEV).to(torch.bfloat16)
    x = torch.randn(rows, K, device=DEV).to(torch.bfloat16)
    ref = dy.float().t() @ x.float()
    dw = torch.full((N, K), 0.5, device=DEV)
    db = torch.full((N,), 0.25, device=DEV)
    ops.linear_wgrad(dy, x, dw, db=db)
    _close(dw, ref + 0.5, 2e-3)
    _close(db, dy.float().sum(0) + 0.25, 1e-4)
    out = torch.full((1, N, K), 7.0, device=DEV)
    ops.gemm(dy, x, out, M=N, N=K, K=rows, lda_m=1, lda_k=N, ldb_k=K, ldb_n=1, ldc=K, beta=0.0)
    _close(out[0], ref, 2e-3)


@pytest.mark.parametrize("rows,N,K", [(20480, 256, 2048), (16384, 2048, 256), (8192, 448, 1792), (14112, 1344, 448),
                                      (40000, 256, 64), (9000, 128, 256), (20000, 112, 448), (3528, 2688, 896),
                                      (3528, 896, 896), (131072, 32, 256), (4100, 72, 136)])
def test_wgrad_deterministic(rows, N, K):
    """long-reduction weight gradients on the deterministic kernel (csrc/gemm_wgrad.hip: per-split fp32
    partial tiles added in fixed order, bias gradient by MFMA against ones): every tile shape it picks
    (256^2, 256x128, 128x256, 128^2, 256x64, 64x256), K tails, partial M / N tiles; against the fp32
    product, accumulate semantics, and bit-identical across repeats with garbage in the workspace"""
    ops = _ops()
    torch.manual_seed(3)
    dy = torch.randn(rows, N, device=DEV).to(torch.bfloat16)
    x = torch.randn(rows, K, device=DEV).to(torch.bfloat16)
    ref = dy.float().t() @ x.float()
    ws = ops.wgrad_workspace(DEV)
    outs = []
    for r in range(4):
        ws.fill_(float("nan") if r % 2 else 1e30)
        dw = torch.full((N, K), 0.5, device=DEV)
        db = torch.full((N,), 0.25, device=DEV)
        ops.linear_wgrad(dy, x, dw, db=db)
        torch.cuda.synchronize()
        outs.append((dw, db))
    _close(outs[0][0], ref + 0.5, 2e-3)
    _close(outs[0][1], dy.float().sum(0) + 0.25, 1e-4)
    for dw, db in outs[1:]:
        assert torch.equal(dw, outs[0][0]) and torch.equal(db, outs[0][1])
    ops.linear_wgrad(dy, x, outs[0][0], accumulate=False, db=outs[0][1])
    _close(outs[0][0], ref, 2e-3)
    _close(outs[0][1], dy.float().sum(0), 1e-4)


def test_split_k_gemm_deterministic():
    """the split-K launches the deterministic weight-gradient kernel does not take (batched, M < 16,
    N < 64) store per-split partial tiles into the workspace and add them in split order
    (gemm_split_reduce_kernel, round 6): bit-identical across repeats with garbage in the workspace,
    against the fp32 product, beta 0 / 1 and the fused row sum.  Cases: the hypernetwork-mask
    gradient dh = g^T up over 104 frames x objects (1 x 32 over 65 536 pixels, frametape._hyper_bw --
    with fp32 atomics its result changed between identical bench-size runs), a 3-batch 40 x 96 over
    20 000, and an 8-row weight gradient with its bias gradient (linear_wgrad, rows = 65 536)"""
    ops = _ops()
    torch.manual_seed(11)
    bf = torch.bfloat16
    ws = ops.wgrad_workspace(DEV)
    g = torch.randn(104, 1, 65536, device=DEV).to(bf)
    up = torch.randn(104, 65536, 32, device=DEV).to(bf)
    a3 = torch.randn(3, 40, 20000, device=DEV).to(bf)
    b3 = torch.randn(3, 20000, 96, device=DEV).to(bf)
    dy = torch.randn(65536, 8, device=DEV).to(bf)
    x = torch.randn(65536, 48, device=DEV).to(bf)
    outs = []
    for r in range(3):
        ws.fill_(float("nan") if r % 2 else 1e30)
        dh = ops.bmm(g, up, torch.full((104, 1, 32), 3.0, device=DEV))
        c3 = ops.bmm(a3, b3, torch.full((3, 40, 96), 0.5, device=DEV), beta=1.0)
        dw = torch.full((8, 48), 0.5, device=DEV)
        db = torch.full((8,), 0.25, device=DEV)
        ops.linear_wgrad(dy, x, dw, db=db)
        torch.cuda.synchronize()
        outs.append((dh, c3, dw, db))
    dh, c3, dw, db = outs[0]
    _close(dh, g.float() @ up.float(), 2e-3)
    _close(c3, a3.float() @ b3.float() + 0.5, 2e-3)
    _close(dw, dy.float().t() @ x.float() + 0.5, 2e-3)
    _close(db, dy.float().sum(0) + 0.25, 1e-4)
    for o in outs[1:]:
        for u, v in zip(o, outs[0]):
            assert torch.equal(u, v)


@pytest.mark.parametrize("rows,H,p", [(93184, 2048, 0.1), (1024, 2048, 0.0), (64, 128, 0.25), (13312, 384, 0.1)])
def test_ffn_bwd_dgrad(rows, H, p):
    """memory-attention FFN backward, input-gradient side, in one launch (csrc/ffn.hip): dH = (dY W2) *
    [hid > 0] / keep and dX = dH W1 against the fp32 products (dX from the kernel's own bf16 dH, as the
    two-GEMM path computes it), the two-GEMM path itself, and bit-identical repeats.  The bench shape
    (93 184 rows, H 2048), one chunk (H 128), a single tile."""
    ops = _ops()
    torch.manual_seed(5)
    bf = torch.bfloat16
    dy = torch.randn(rows, 256, device=DEV).to(bf)
    w2 = (torch.randn(256, H, device=DEV) / math.sqrt(H)).to(bf)
    w1 = (torch.randn(H, 256, device=DEV) / 16).to(bf)
    hid = torch.relu(torch.randn(rows, H, device=DEV)).to(bf)
    if p > 0:  # dropped elements are zeros of hid too
        hid = hid * (torch.rand(rows, H, device=DEV) >= p).to(bf)
    alpha = 1.0 / (1.0 - p)
    dh, dx = ops.ffn_bwd_dgrad(dy, w2, w1, hid, alpha)
    torch.cuda.synchronize()
    ref_h = alpha * (dy.float() @ w2.float()) * (hid > 0).float()
    _close(dh.float(), ref_h, 8e-3)
    assert not dh[hid == 0].any()
    _close(dx.float(), dh.float() @ w1.float(), 8e-3)
    # the two-GEMM path
    dh2 = ops.linear_dgrad(dy, w2, pre=hid, act="relu", alpha=alpha)
    dx2 = ops.linear_dgrad(dh2, w1)
    _close(dh.float(), dh2.float(), 8e-3)
    _close(dx.float(), dx2.float(), 8e-3)
    for _ in range(2):
        dh3, dx3 = ops.ffn_bwd_dgrad(dy, w2, w1, hid, alpha)
        assert torch.equal(dh3, dh) and torch.equal(dx3, dx)
    # strided dY rows (a view of a wider buffer)
    wide = torch.zeros(rows, 264, device=DEV, dtype=bf)
    wide[:, :256] = dy
    dh4, dx4 = ops.ffn_bwd_dgrad(wide[:, :256], w2, w1, hid, alpha)
    assert torch.equal(dh4, dh) and torch.equal(dx4, dx)


@pytest.mark.parametrize("rows,H,p,idx", [(13312, 2048, 0.1, 13312 * 2048 * 3), (1024, 2048, 0.0, 0),
                                          (64, 1024, 0.25, 7), (93184, 2048, 0.1, 0)])
def test_ffn_fwd(rows, H, p, idx):
    """memory-attention FFN forward in one launch (csrc/ffn.hip ffn_fwd_kernel) against the two GEMM
    launches it replaces with the same dropout seeds and element offsets (an odd offset takes the
    per-element hash path): the saved hid and the output within bf16 rounding, the dropout / ReLU
    zeros identical, bit-identical repeats"""
    ops = _ops()
    torch.manual_seed(9)
    bf = torch.bfloat16
    x = torch.randn(rows, 256, device=DEV).to(bf)
    w1 = (torch.randn(H, 256, device=DEV) / 16).to(bf)
    b1 = torch.randn(H, device=DEV) * 0.1
    w2 = (torch.randn(256, H, device=DEV) / math.sqrt(H)).to(bf)
    b2 = torch.randn(256, device=DEV) * 0.1
    s1, s2 = 0x1234567, 0x89ABCDEF
    hid, y = ops.ffn_fwd(x, w1, b1, w2, b2, p, s1, idx, s2, idx + 1)
    hid_r = ops.linear(x, w1, b1, act="relu", drop_p=p, seed=s1, drop_idx0=idx)
    y_r = ops.linear(hid_r, w2, b2, drop_p=p, seed=s2, drop_idx0=idx + 1)
    torch.cuda.synchronize()
    assert torch.equal(hid == 0, hid_r == 0)
    _close(hid.float(), hid_r.float(), 8e-3)
    _close(y.float(), y_r.float(), 8e-3)
    if p > 0:
        assert torch.equal(y == 0, y_r == 0)
    pos = (x.float() @ w1.float().t() + b1) > 1e-2  # clearly positive pre-activations: dropped at rate p
    assert abs((hid[pos] == 0).float().mean().item() - p) < 0.03
    hid2, y2 = ops.ffn_fwd(x, w1, b1, w2, b2, p, s1, idx, s2, idx + 1)
    assert torch.equal(hid2, hid) and torch.equal(y2, y)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,H,W,C,ws",[(8, 32, 32, 1344, 14), (8, 16, 16, 2688, 7), (2, 9, 13, 48, 4), (1, 8, 8, 16, 8)])
def test_window_pad(dtype, B, H, W, C, ws):
    """partition of a projection's output with bias rows at the padded positions (Hiera's padded windows,
    csrc/elementwise.hip window_pad_vec_kernel) against zero-pad + partition + bias fill in torch, and
    its bias gradient (the padded rows' column sums, window_pad_colsum_kernel) against torch"""
    ops = _ops()
    ops.wgrad_workspace(DEV)  # the deterministic-reduction workspace (SAM2Model.load registers it)
    torch.manual_seed(7)
    x = torch.randn(B, H, W, C, device=DEV).to(dtype)
    bias = torch.randn(C, device=DEV)
    nh, nw = -(-H // ws), -(-W // ws)
    pad = torch.zeros(B, nh * ws, nw * ws, C, device=DEV, dtype=dtype)
    pad[:] = bias.to(dtype)
    pad[:, :H, :W] = x
    ref = pad.view(B, nh, ws, nw, ws, C).permute(0, 1, 3, 2, 4, 5).reshape(B * nh * nw, ws, ws, C)
    out = ops.window_pad(x, ws, bias)
    assert torch.equal(out, ref)
    g = torch.randn(B * nh * nw, ws, ws, C, device=DEV).to(dtype)
    gp = g.view(B, nh, nw, ws, ws, C).permute(0, 1, 3, 2, 4, 5).reshape(B, nh * ws, nw * ws, C).float()
    mask = torch.ones(nh * ws, nw * ws, dtype=torch.bool, device=DEV)
    mask[:H, :W] = False
    want = gp[:, mask].sum((0, 1)) + 0.5
    got = torch.full((C,), 0.5, device=DEV)
    ops.window_pad_colsum(g, ws, B, H, W, got)
    _close(got, want, 1e-5)
    again = torch.full((C,), 0.5, device=DEV)
    ops.window_pad_colsum(g, ws, B, H, W, again)
    assert torch.equal(again, got)


@pytest.mark.parametrize("compute", ["fp32", "bf16"])
@pytest.mark.parametrize("dim,heads,ws,HW", [(448, 8, 14, 32), (896, 8, 7, 16)])
def test_hiera_padded_window_block(compute, dim, heads, ws, HW, monkeypatch):
    """a Hiera block whose windows need padding (B+ at 512^2: stage 3, 32 -> 42; stage 4, 16 -> 21) with the
    qkv projection over the real tokens + bias-row partition (hieradet.py, S2H_HIERA_PAD_QKV=1) against the
    reference order (zero-pad the normed input, project every padded row; =0): the block output
    bit-identical, every parameter gradient within summation order"""
    from sam2_video.kernels.arena import ParamArena
    from sam2_video.model.modeling.backbones.hieradet import MultiScaleBlock
    _ops().wgrad_workspace(DEV)
    torch.manual_seed(11)
    blk = MultiScaleBlock(dim, dim, heads, window_size=ws)
    for p in blk.parameters():
        p.data = torch.randn_like(p) * 0.05
    cd = torch.float32 if compute == "fp32" else torch.bfloat16
    arena = ParamArena(list(blk.named_parameters()), [n for n, _ in blk.named_parameters()], cd, DEV)
    x0 = torch.randn(4, HW, HW, dim, device=DEV).to(cd)
    res = {}
    for flag in ("0", "1"):
        monkeypatch.setenv("S2H_HIERA_PAD_QKV", flag)
        arena.grad.zero_()
        x = x0.clone().requires_grad_(True)
        y = blk(x)
        g = torch.randn(y.shape, device=DEV, generator=torch.Generator(DEV).manual_seed(3)).to(cd)
        y.backward(g)
        torch.cuda.synchronize()
        res[flag] = (y.detach().clone(), x.grad.clone(), arena.grad.clone())
    assert torch.equal(res["0"][0], res["1"][0])
    tol = 1e-5 if compute == "fp32" else 1e-2
    _close(res["1"][1], res["0"][1], tol)
    for n in arena.grad_names:
        o, k = arena.offsets[n], blk.get_parameter(n).numel()
        _close(res["1"][2][o:o + k], res["0"][2][o:o + k], tol)


@pytest.mark.parametrize("compute", ["fp32", "bf16"])
def test_hiera_stage_window_order(compute, monkeypatch):
    """the Hiera trunk with its whole-window stages kept in window order between one partition and one
    unpartition (S2H_HIERA_WIN_STAGE=1; B+ at 256^2: stages 1 and 2) against a partition / unpartition
    around every block's attention (=0, hieradet.py:146,161): every stage output bit-identical (the same
    per-token ops and per-window attention), input and parameter gradients within summation order"""
    from sam2_video.kernels.arena import ParamArena
    from sam2_video.model.modeling.backbones.hieradet import Hiera
    _ops().wgrad_workspace(DEV)
    torch.manual_seed(12)
    trunk = Hiera(embed_dim=112, num_heads=2, stages=(2, 3, 16, 3), global_att_blocks=(12, 16, 20))
    assert trunk.window_stages(64, 64) == {0: (1, 8), 2: (4, 8)}
    for p in trunk.parameters():
        p.data = torch.randn_like(p) * 0.05
    cd = torch.float32 if compute == "fp32" else torch.bfloat16
    arena = ParamArena(list(trunk.named_parameters()), [n for n, _ in trunk.named_parameters()], cd, DEV)
    x0 = torch.randn(2, 256, 256, 3, device=DEV).to(cd)
    res = {}
    for flag in ("0", "1"):
        monkeypatch.setenv("S2H_HIERA_WIN_STAGE", flag)
        arena.grad.zero_()
        outs = trunk(x0)
        gen = torch.Generator(DEV).manual_seed(5)
        gs = [torch.randn(o.shape, device=DEV, generator=gen).to(cd) for o in outs]
        torch.autograd.backward(outs, gs)
        torch.cuda.synchronize()
        res[flag] = ([o.detach().clone() for o in outs], arena.grad.clone())
    for a, b in zip(res["0"][0], res["1"][0]):
        assert torch.equal(a, b)
    tol = 1e-5 if compute == "fp32" else 2e-2
    for n in arena.grad_names:
        o, k = arena.offsets[n], trunk.get_parameter(n).numel()
        _close(res["1"][1][o:o + k], res["0"][1][o:o + k], tol)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("rows,cols", [(131072, 112), (13312, 2048), (5, 24), (1000, 37), (70000, 256), (3, 4096)])
def test_colsum_shapes(dtype, rows, cols):
    ops = _ops()
    torch.manual_seed(2)
    x = torch.randn(rows, cols, device=DEV).to(dtype)
    out = torch.full((cols,), 1.0, device=DEV)
    ops.colsum(x, out)  # accumulate
    _close(out, x.float().sum(0) + 1.0, 1e-4)
    ops.colsum(x, out, accumulate=False)
    _close(out, x.float().sum(0), 1e-4)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_memory_pos_and_segmented_colsum(dtype):
    """memory positions of every slot in one launch (s2h_memory_pos) == the per-slot broadcast adds;
    segmented column sums (s2h_colsum_seg) == per-segment colsum, incl. two segments into one row"""
    ops = _ops()
    torch.manual_seed(3)
    L, C = 4096, 64
    pos = torch.randn(L, C, device=DEV).to(dtype)
    tpos = torch.randn(7, C, device=DEV).to(dtype)
    idx = [6, 0, 3, 5, 1]
    out = torch.empty(len(idx) * L, C, device=DEV, dtype=dtype)
    ops.memory_pos(pos, tpos, idx, out)
    ref = torch.cat([ops.add_bcast(pos, tpos[i], out=torch.empty_like(pos)) for i in idx])
    assert torch.equal(out, ref)
    x = torch.randn(9 * 1000, C, device=DEV).to(dtype)
    offs, dsts = [0, 1000, 3000, 7000, 5000], [2, 0, 2, 4, 1]
    got = torch.full((5, C), 0.5, device=DEV)
    ops.colsum_seg(x, 1000, offs, dsts, got)
    want = torch.full((5, C), 0.5, device=DEV)
    for o, d in zip(offs, dsts):
        want[d] += x[o:o + 1000].float().sum(0)
    _close(got, want, 1e-5)


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-5), (torch.bfloat16, 1e-2)])
def test_bmm_layouts(dtype, tol):
    ops = _ops()
    a = torch.randn(3, 37, 50, device=DEV).to(dtype)
    b = torch.randn(3, 50, 70, device=DEV).to(dtype)
    out = torch.empty(3, 37, 70, device=DEV, dtype=dtype)
    ops.bmm(a, b, out)
    _close(out, a.float() @ b.float(), tol)
    bt = torch.randn(3, 70, 50, device=DEV).to(dtype)
    ops.bmm(a, bt, out, trans_b=True)
    _close(out, a.float() @ bt.float().transpose(1, 2), tol)
    at = torch.randn(3, 50, 37, device=DEV).to(dtype).transpose(1, 2)  # M-contiguous A
    ops.bmm(at, b, out)
    _close(out, at.float() @ b.float(), tol)


def _ref_attn(q, k, v, scale):
    # q [B, Lq, H, D]
    qh, kh, vh = (t.float().transpose(1, 2) for t in (q, k, v))
    s = (qh @ kh.transpose(-1, -2)) * scale
    p = s.softmax(-1)
    return (p @ vh).transpose(1, 2), torch.logsumexp(s, -1)


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 5e-5), (torch.bfloat16, 2e-2)])
@pytest.mark.parametrize("B,H,Lq,Lk,D", [(2, 2, 64, 64, 56), (3, 1, 16, 64, 56), (2, 8, 8, 100, 16),
                                         (2, 8, 100, 8, 16), (1, 8, 7, 7, 32), (2, 1, 256, 1028, 256),
                                         (1, 4, 196, 196, 96), (1, 2, 49, 196, 72), (13, 1, 70, 130, 256),
                                         # decoder token<->image shapes: few-query / few-key kernels
                                         (13, 8, 8, 1024, 16), (13, 8, 1024, 8, 16), (2, 3, 5, 300, 32),
                                         (2, 3, 300, 5, 32), (1, 2, 16, 1000, 64), (1, 2, 1000, 16, 64)])
def test_attention_fwd_bwd(dtype, tol, B, H, Lq, Lk, D):
    ops = _ops()
    torch.manual_seed(1)
    q = torch.randn(B, Lq, H, D, device=DEV).to(dtype)
    k = torch.randn(B, Lk, H, D, device=DEV).to(dtype)
    v = torch.randn(B, Lk, H, D, device=DEV).to(dtype)
    scale = 1.0 / math.sqrt(D)
    o = torch.empty_like(q)
    lse = torch.empty(B, H, Lq, device=DEV)
    ops.attn_fwd(q, k, v, o, lse, scale)
    qr, kr, vr = (t.float().clone().requires_grad_(True) for t in (q, k, v))
    ro, rl = _ref_attn(qr, kr, vr, scale)
    _close(o, ro, tol)
    _close(lse, rl, tol)
    do = torch.randn_like(q)
    ro.backward(do.float())
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    ops.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, scale)
    _close(dq, qr.grad, 3 * tol)
    _close(dk, kr.grad, 3 * tol)
    _close(dv, vr.grad, 3 * tol)


@pytest.mark.parametrize("B,H,Lq,Lk,D", [(256, 4, 16, 16, 56), (512, 2, 4, 16, 56), (128, 2, 16, 64, 56),
                                         (64, 2, 64, 64, 56), (16, 8, 49, 49, 56), (13, 8, 8, 8, 32),
                                         (3, 2, 7, 5, 40), (2, 3, 33, 17, 64), (5, 1, 1, 2, 8), (4, 2, 17, 64, 24),
                                         # long query side, few keys (forward on the window kernel)
                                         (13, 8, 1024, 8, 16), (2, 2, 130, 40, 64)])
def test_small_window_attention(B, H, Lq, Lk, D):
    """Hiera window / pooled-query shapes (Lq, Lk <= 64) on the whole-instance kernels
    (attention.hip attn_win_*): forward, LSE and the one-launch backward against the fp32
    reference and against the tile kernels (s2h_attn_win(0)) on the same bf16 inputs"""
    from sam2_video.kernels import _lib
    ops = _ops()
    torch.manual_seed(6)
    bf = torch.bfloat16
    q = torch.randn(B, Lq, H, D, device=DEV).to(bf)
    k = torch.randn(B, Lk, H, D, device=DEV).to(bf)
    v = torch.randn(B, Lk, H, D, device=DEV).to(bf)
    do = torch.randn(B, Lq, H, D, device=DEV).to(bf)
    scale = 1.0 / math.sqrt(D)
    res = {}
    for on in (1, 0):
        prev = _lib.lib().s2h_attn_win(on)
        try:
            o = torch.full_like(q, float("nan"))
            lse = torch.full((B, H, Lq), float("nan"), device=DEV)
            ops.attn_fwd(q, k, v, o, lse, scale)
            dq, dk, dv = (torch.full_like(t, float("nan")) for t in (q, k, v))
            ops.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, scale)
            res[on] = (o, lse, dq, dk, dv)
        finally:
            _lib.lib().s2h_attn_win(prev)
    qr, kr, vr = (t.float().clone().requires_grad_(True) for t in (q, k, v))
    ro, rl = _ref_attn(qr, kr, vr, scale)
    ro.backward(do.float())
    o, lse, dq, dk, dv = res[1]
    for t in res[1]:
        assert not torch.isnan(t.float()).any()
    _close(o, ro, 2e-2)
    _close(lse, rl, 2e-2)
    _close(dq, qr.grad, 6e-2)
    _close(dk, kr.grad, 6e-2)
    _close(dv, vr.grad, 6e-2)
    for a_, b_ in zip(res[1], res[0]):  # same bf16 rounding points as the tile kernels
        _close(a_, b_, 3e-2)


@pytest.mark.parametrize("B,H,Lq,Lk,D", [(13, 1, 1024, 7196, 256), (13, 1, 1024, 1024, 256), (2, 2, 1024, 1028, 128),
                                         (2, 4, 300, 77, 64), (1, 1, 1000, 1031, 256), (3, 1, 128, 40, 256),
                                         # Hiera head dim 56 (and 40) in the padded 64 image
                                         (2, 2, 196, 196, 56), (1, 8, 1024, 1024, 56), (3, 2, 130, 300, 40),
                                         (2, 4, 256, 200, 64),
                                         # Hiera-L head dim 72 (and 96, 120) in the padded 128 image
                                         (2, 2, 256, 256, 72), (1, 4, 4096, 4096, 72), (1, 2, 300, 700, 96),
                                         (2, 1, 130, 200, 120)])
def test_flash_forward_matches_reference(B, H, Lq, Lk, D):
    """bf16 long-sequence path (flash.hip, flash_bwd.hip): key-split partials + combine, ragged
    tails, head dims <= 64 padded to the 64 image."""
    ops = _ops()
    torch.manual_seed(4)
    q = torch.randn(B, Lq, H, D, device=DEV).to(torch.bfloat16)
    k = torch.randn(B, Lk, H, D, device=DEV).to(torch.bfloat16)
    v = torch.randn(B, Lk, H, D, device=DEV).to(torch.bfloat16)
    scale = 1.0 / math.sqrt(D)
    o = torch.empty_like(q)
    lse = torch.empty(B, H, Lq, device=DEV)
    ops.attn_fwd(q, k, v, o, lse, scale)
    qr, kr, vr = (t.float().clone().requires_grad_(True) for t in (q, k, v))
    ro, rl = _ref_attn(qr, kr, vr, scale)
    _close(o, ro, 2e-2)
    _close(lse, rl, 1e-3)
    do = torch.randn_like(q)
    ro.backward(do.float())
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    ops.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, scale)
    _close(dq, qr.grad, 4e-2)
    _close(dk, kr.grad, 4e-2)
    _close(dv, vr.grad, 4e-2)


@pytest.mark.parametrize("target", [1, 64, 256, 4096])
def test_flash_forward_split_counts(target):
    """Every key-split count (s2h_attn_config bits 8+) gives the reference output."""
    from sam2_video.kernels._lib import lib
    ops = _ops()
    torch.manual_seed(6)
    B, H, Lq, Lk, D = 2, 1, 512, 2000, 256
    q, k, v = (torch.randn(B, L, H, D, device=DEV).to(torch.bfloat16) for L in (Lq, Lk, Lk))
    o = torch.empty_like(q)
    lse = torch.empty(B, H, Lq, device=DEV)
    prev = lib().s2h_attn_config(1 | (target << 8))
    try:
        ops.attn_fwd(q, k, v, o, lse, 0.0625)
    finally:
        lib().s2h_attn_config(prev)
    ro, rl = _ref_attn(q.float(), k.float(), v.float(), 0.0625)
    _close(o, ro, 2e-2)
    _close(lse, rl, 1e-3)


@pytest.mark.parametrize("kind,B,H,Lq,Lk,D,p,target", [
    ("vfold", 13, 1, 1024, 3084, 256, 0.1, 256), ("vfold", 3, 1, 300, 1028, 256, 0.1, 256),
    ("vfold", 2, 1, 1000, 700, 256, 0.0, 64), ("vfold", 13, 1, 1024, 7196, 256, 0.1, 4096),
    ("plain", 1, 8, 1024, 1024, 56, 0.0, 256), ("plain", 2, 2, 196, 196, 56, 0.0, 64),
    ("plain", 2, 4, 300, 77, 64, 0.1, 256), ("plain", 1, 4, 4096, 4096, 72, 0.0, 256),
    ("plain", 2, 1, 130, 200, 120, 0.1, 64)])
def test_flash_forward_query_sets_bit_identical(kind, B, H, Lq, Lk, D, p, target):
    """the forward with two 16-query sets per wave (s2h_flash_fwd_sets, default for the V-fold
    cross-attention and head dims <= 128: every K / V fragment read from LDS feeds two MFMAs) gives
    the one-set kernel's bits -- output, log-sum-exp and dropout keep bitmap -- on one key split,
    across ragged query / key tails and padded head dims; with key splits (whose count follows the
    workgroup count, so differs between the two forms) the outputs agree to the combine's rounding"""
    from sam2_video.kernels._lib import lib
    ops = _ops()
    torch.manual_seed(11)
    bf = torch.bfloat16
    q = (torch.randn(B, Lq, H, D, device=DEV) * 0.5).to(bf)
    k = (torch.randn(B, Lk, H, D, device=DEV) * 0.5).to(bf)
    v = torch.randn(B, Lk, H, 64 if kind == "vfold" else D, device=DEV).to(bf)

    def run(qs, tgt):
        prev_t = lib().s2h_attn_config(1 | (tgt << 8))
        prev = lib().s2h_flash_fwd_sets(qs)
        try:
            o = torch.full((B, Lq, H, 72 if kind == "vfold" else D), 7.0, device=DEV, dtype=bf)
            lse = torch.full((B, H, Lq), 7.0, device=DEV)
            # (a keep bitmap only for the 256-wide heads whose backward reads it)
            keep = (torch.zeros(ops.keep_words(B, H, Lq, Lk), device=DEV, dtype=torch.int32)
                    if p > 0 and kind == "vfold" else None)
            if kind == "vfold":
                ops.attn_fwd_vfold(q, k, v, o, lse, 0.0625, p, 5, idx0=6, keep=keep)
            else:
                ops.attn_fwd(q, k, v, o, lse, D ** -0.5, p, 5, idx0=6, keep=keep)
            torch.cuda.synchronize()
            return o, lse, keep
        finally:
            lib().s2h_flash_fwd_sets(prev)
            lib().s2h_attn_config(prev_t)
    (o1, l1, k1), (o2, l2, k2) = run(0x11, 1), run(0x22, 1)
    assert torch.equal(o1, o2), (o1.float() - o2.float()).abs().max().item()
    assert torch.equal(l1, l2)
    (o3, l3, k3), (o4, l4, k4) = run(0x11, target), run(0x22, target)
    _close(o4, o3.float(), 2e-2)
    _close(l4, l3, 1e-4)
    _close(o4, o1.float(), 2e-2)
    if k1 is not None:
        assert torch.equal(k1, k2) and torch.equal(k1, k3) and torch.equal(k1, k4)


def test_flash_dropout_matches_generic_kernel():
    """Same counter-hash dropout mask in the flash and the generic forward (the backward
    regenerates it), so both produce the same output up to bf16 rounding."""
    from sam2_video.kernels._lib import lib
    ops = _ops()
    torch.manual_seed(5)
    B, H, Lq, Lk, D = 2, 1, 256, 700, 256
    q, k, v = (torch.randn(B, L, H, D, device=DEV).to(torch.bfloat16) for L in (Lq, Lk, Lk))
    o1, o2 = torch.empty_like(q), torch.empty_like(q)
    l1, l2 = torch.empty(B, H, Lq, device=DEV), torch.empty(B, H, Lq, device=DEV)
    ops.attn_fwd(q, k, v, o1, l1, 0.0625, p_drop=0.1, seed=77)
    do = torch.randn_like(q)
    g1 = [torch.empty_like(t) for t in (q, k, v)]
    g2 = [torch.empty_like(t) for t in (q, k, v)]
    ops.attn_bwd(q, k, v, o1, do, l1, *g1, 0.0625, p_drop=0.1, seed=77)
    prev = lib().s2h_attn_config(0)
    try:
        ops.attn_fwd(q, k, v, o2, l2, 0.0625, p_drop=0.1, seed=77)
        ops.attn_bwd(q, k, v, o2, do, l2, *g2, 0.0625, p_drop=0.1, seed=77)
    finally:
        lib().s2h_attn_config(prev)
    _close(o1, o2, 2e-2)
    _close(l1, l2, 1e-4)
    for a_, b_ in zip(g1, g2):
        _close(a_, b_, 3e-2)


def test_attention_strided_qkv():
    """q/k/v read in place from a fused [B, L, 3, H, d] qkv projection (Hiera)."""
    ops = _ops()
    B, L, H, d = 4, 64, 2, 56
    qkv = torch.randn(B, L, 3, H, d, device=DEV)
    q, k, v = qkv.unbind(2)
    o = torch.empty(B, L, H, d, device=DEV)
    lse = torch.empty(B, H, L, device=DEV)
    ops.attn_fwd(q, k, v, o, lse, d ** -0.5)
    ro, _ = _ref_attn(q, k, v, d ** -0.5)
    _close(o, ro, 5e-5)


@pytest.mark.parametrize("Lq,Lk", [(40, 40), (8, 300), (300, 8)])
def test_attention_dropout_consistent(Lq, Lk):
    """dropout mask regenerated in backward: finite-difference check of the dropped attention."""
    ops = _ops()
    torch.manual_seed(2)
    B, H, D = 1, 1, 32
    q = torch.randn(B, Lq, H, D, device=DEV, dtype=torch.float64).float()
    k = torch.randn(B, Lk, H, D, device=DEV).float()
    v = torch.randn(B, Lk, H, D, device=DEV).float()
    o = torch.empty_like(q)
    lse = torch.empty(B, H, Lq, device=DEV)
    ops.attn_fwd(q, k, v, o, lse, 0.2, p_drop=0.3, seed=1234)
    o2 = torch.empty_like(q)
    ops.attn_fwd(q, k, v, o2, lse, 0.2, p_drop=0.3, seed=1234)
    assert torch.equal(o, o2)
    do = torch.randn_like(o)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    ops.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, 0.2, p_drop=0.3, seed=1234)
    # directional derivative along random dv direction: <do, dO/dv . e> == <dv, e>
    e = torch.randn_like(v) * 1e-2
    op = torch.empty_like(o)
    ops.attn_fwd(q, k, v + e, op, lse.clone(), 0.2, p_drop=0.3, seed=1234)
    lhs = ((op - o) * do).sum().item()
    rhs = (dv * e).sum().item()
    assert abs(lhs - rhs) <= 1e-3 * max(1.0, abs(rhs))
    eq = torch.randn_like(q) * 1e-3
    ops.attn_fwd(q + eq, k, v, op, lse.clone(), 0.2, p_drop=0.3, seed=1234)
    lhs = ((op - o) * do).sum().item()
    rhs = (dq * eq).sum().item()
    assert abs(lhs - rhs) <= 2e-2 * max(1e-2, abs(rhs))


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 1e-2)])
@pytest.mark.parametrize("rows,C", [(1, 112), (1000, 256), (37, 896), (513, 64), (9, 1152), (77, 4), (50, 20),
                                    (4099, 32), (13312, 256), (300, 448)])
def test_layernorm(dtype, tol, rows, C):
    ops = _ops()
    x = torch.randn(rows, C, device=DEV).to(dtype)
    g = torch.randn(C, device=DEV)
    b = torch.randn(C, device=DEV)
    y, mu, rs = ops.layernorm_fwd(x, g, b, 1e-6)
    xr = x.float().clone().requires_grad_(True)
    gr = g.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    yr = torch.nn.functional.layer_norm(xr, (C,), gr, br, 1e-6)
    _close(y, yr, tol)
    dy = torch.randn(rows, C, device=DEV).to(dtype)
    yr.backward(dy.float())
    dg = torch.zeros(C, device=DEV)
    db = torch.zeros(C, device=DEV)
    dx = ops.layernorm_bwd(x, dy, g, mu, rs, dgamma=dg, dbeta=db)
    _close(dx, xr.grad, 3 * tol)
    _close(dg, gr.grad, 3 * tol * max(1.0, rows / 1000) ** 0.5)
    _close(db, br.grad, 3 * tol * max(1.0, rows / 1000) ** 0.5)
    # fused residual-stream gradient (dx = LN'(dy) + dres) and accumulation into existing weight grads
    dres = torch.randn(rows, C, device=DEV).to(dtype)
    dx2 = ops.layernorm_bwd(x, dy, g, mu, rs, dres=dres, dgamma=dg, dbeta=db)
    _close(dx2, xr.grad + dres.float(), 3 * tol)
    _close(dg, 2 * gr.grad, 6 * tol * max(1.0, rows / 1000) ** 0.5)
    a = torch.randn(rows, C, device=DEV).to(dtype)
    xs = torch.empty_like(x)
    y2, _, _ = ops.layernorm_fwd(x, g, b, 1e-6, add=a, xsum=xs)
    _close(xs, x.float() + a.float(), tol)
    _close(y2, torch.nn.functional.layer_norm(xs.float(), (C,), g, b, 1e-6), tol)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_maxpool2_vector_path_matches_torch(dtype):
    """the 16-B maxpool forms (round 6; C a multiple of 8 / 4, strided pixels): values with many ties and a
    few NaNs, odd H / W -- the same pooled values and the same gradient routing (first maximum of the
    window scan, NaN wins) as torch's max_pool2d"""
    ops = _ops()
    torch.manual_seed(5)
    full = torch.randint(-3, 4, (3, 17, 14, 64), device=DEV).to(dtype)
    full.view(-1)[torch.randperm(full.numel(), device=DEV)[:40]] = float("nan")
    x = full[..., :48]  # pixel stride 64
    y = ops.maxpool2(x)
    xr = x.float().permute(0, 3, 1, 2).contiguous().requires_grad_(True)
    ref = torch.nn.functional.max_pool2d(xr, 2)
    torch.testing.assert_close(y.float(), ref.permute(0, 2, 3, 1), rtol=0, atol=0, equal_nan=True)
    g = torch.randn(y.shape, device=DEV).to(dtype)
    ref.backward(g.float().permute(0, 3, 1, 2))
    dx = torch.full_like(x, 7.0)
    ops.maxpool2_bwd(x, g.contiguous(), dx)
    exp = xr.grad.permute(0, 2, 3, 1)
    torch.testing.assert_close(dx[:, :16, :14].float(), exp[:, :16, :14], rtol=0, atol=0)
    assert bool((dx[:, 16] == 7.0).all())  # the odd last row is outside every window: untouched


def test_elementwise_misc():
    ops = _ops()
    x = torch.randn(2, 10, 12, 6, device=DEV)
    y = ops.maxpool2(x)
    ref = torch.nn.functional.max_pool2d(x.permute(0, 3, 1, 2), 2).permute(0, 2, 3, 1)
    _close(y, ref, 0)
    xr = x.clone().requires_grad_(True)
    torch.nn.functional.max_pool2d(xr.permute(0, 3, 1, 2), 2).permute(0, 2, 3, 1).backward(torch.ones_like(y))
    dx = torch.empty_like(x)
    ops.maxpool2_bwd(x, torch.ones_like(y), dx)
    _close(dx, xr.grad, 0)
    # window partition / unpartition with padding
    x = torch.randn(2, 9, 11, 5, device=DEV)
    win = ops.window_partition(x, 4)
    xp = torch.nn.functional.pad(x, (0, 0, 0, 1, 0, 3))
    ref = xp.view(2, 3, 4, 3, 4, 5).permute(0, 1, 3, 2, 4, 5).reshape(-1, 4, 4, 5)
    _close(win, ref, 0)
    back = ops.window_unpartition(win, 4, 2, 9, 11)
    _close(back, x, 0)
    # bilinear
    lo = torch.randn(3, 16, 16, device=DEV)
    hi = ops.bilinear(lo, 64, 64)
    ref = torch.nn.functional.interpolate(lo[:, None], size=(64, 64), mode="bilinear", align_corners=False)[:, 0]
    _close(hi, ref, 1e-6)
    lr = lo.clone().requires_grad_(True)
    g = torch.randn(3, 64, 64, device=DEV)
    torch.nn.functional.interpolate(lr[:, None], size=(64, 64), mode="bilinear", align_corners=False)[:, 0].backward(g)
    _close(ops.bilinear_bwd(g, 16, 16), lr.grad, 1e-5)
    # nearest up2 add + its backward
    lat = torch.randn(2, 8, 8, 4, device=DEV)
    prev = torch.randn(2, 4, 4, 4, device=DEV)
    out = ops.up2_add(lat, prev)
    ref = lat + prev.repeat_interleave(2, 1).repeat_interleave(2, 2)
    _close(out, ref, 0)
    dp = torch.empty_like(prev)
    ops.pool2_sum(out, dp)
    _close(dp, out.view(2, 4, 2, 4, 2, 4).sum((2, 4)), 1e-6)
    # colsum
    t = torch.randn(1000, 33, device=DEV)
    cs = torch.zeros(33, device=DEV)
    ops.colsum(t, cs)
    _close(cs, t.sum(0), 1e-5)


def test_im2col_conv_matches_torch():
    ops = _ops()
    x = torch.randn(2, 17, 19, 3, device=DEV)
    w = torch.randn(8, 3, 7, 7, device=DEV)
    b = torch.randn(8, device=DEV)
    col, Ho, Wo = ops.im2col(x, 7, 7, 4, 3)
    y = ops.linear(col, w.reshape(8, -1), b).view(2, Ho, Wo, 8)
    ref = _cpu_conv(torch.nn.functional.conv2d, x.permute(0, 3, 1, 2), w, b, stride=4, padding=3).permute(0, 2, 3, 1)
    _close(y, ref, 2e-5)
    wd = torch.randn(6, 1, 7, 7, device=DEV)
    xd = torch.randn(2, 9, 9, 6, device=DEV)
    yd = ops.dwconv(xd, wd, b[:6], 3)
    ref = _cpu_conv(torch.nn.functional.conv2d, xd.permute(0, 3, 1, 2), wd, b[:6], padding=3, groups=6).permute(0, 2, 3, 1)
    _close(yd, ref, 2e-5)


@pytest.mark.parametrize("B,H,W,C,k,s,p,pad8", [(8, 512, 512, 3, 7, 4, 3, True), (2, 17, 19, 3, 7, 4, 3, True),
                                               (13, 32, 32, 16, 4, 4, 0, False), (2, 9, 7, 5, 3, 2, 1, False)])
def test_im2col_bf16_equals_unfold(B, H, W, C, k, s, p, pad8):
    """bf16 im2col (the 8-columns-per-lane kernel when the row pitch allows, round 6) is an exact copy:
    equal to torch's unfold of the NCHW image, column order (c, ky, kx), padding rows zero"""
    ops = _ops()
    torch.manual_seed(15)
    x = torch.randn(B, H, W, C, device=DEV).to(torch.bfloat16)
    col, Ho, Wo = ops.im2col(x, k, k, s, p, pad8=pad8)
    ref = torch.nn.functional.unfold(x.permute(0, 3, 1, 2).float(), k, padding=p, stride=s)  # [B, C*k*k, L]
    ref = ref.transpose(1, 2).reshape(B * Ho * Wo, C * k * k).to(torch.bfloat16)
    assert torch.equal(col, ref)
    if pad8 and col.stride(0) != col.shape[1]:  # the padding columns of the pitch are zero
        full = col.as_strided((col.shape[0], col.stride(0)), (col.stride(0), 1))
        assert not full[:, col.shape[1]:].float().abs().sum().item()


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-5), (torch.bfloat16, 1e-2)])
@pytest.mark.parametrize("B,H,W,C", [(13, 32, 32, 256), (2, 7, 45, 128), (13, 64, 64, 256), (1, 5, 3, 64)])
def test_dwconv_vectorised(dtype, tol, B, H, W, C):
    ops = _ops()
    torch.manual_seed(3)
    x = torch.randn(B, H, W, C, device=DEV).to(dtype)
    w = torch.randn(C, 1, 7, 7, device=DEV)
    b = torch.randn(C, device=DEV)
    y = ops.dwconv(x, w, b, 3)
    ref = _cpu_conv(torch.nn.functional.conv2d, x.float().permute(0, 3, 1, 2), w, b, padding=3, groups=C).permute(0, 2, 3, 1)
    _close(y, ref, tol)


def test_convt2():
    ops = _ops()
    B, H, W, Ci, Co = 2, 5, 6, 8, 4
    x = torch.randn(B, H, W, Ci, device=DEV)
    w = torch.randn(Ci, Co, 2, 2, device=DEV)
    b = torch.randn(Co, device=DEV)
    Y = torch.empty(B * H * W, Co * 4, device=DEV)
    x2 = x.reshape(-1, Ci)
    ops.gemm(x2, w, Y, M=B * H * W, N=Co * 4, K=Ci, lda_m=Ci, lda_k=1, ldb_k=Co * 4, ldb_n=1, ldc=Co * 4)
    out = ops.convt2_scatter(Y, B, H, W, Co, bias=b)
    ref = _cpu_conv(torch.nn.functional.conv_transpose2d, x.permute(0, 3, 1, 2), w, b, stride=2).permute(0, 2, 3, 1)
    _close(out, ref, 2e-5)
    dY = ops.convt2_gather(out, B, H, W, Co)
    Y2 = torch.empty_like(Y)
    Y2.copy_(dY)
    out2 = ops.convt2_scatter(Y2, B, H, W, Co)
    _close(out2, out, 0)


def test_rope_roundtrip():
    ops = _ops()
    Bt, L, D = 3, 20, 8
    x = torch.randn(Bt, L, D, device=DEV)
    ang = torch.rand(10, D // 2, device=DEV) * 6
    cos, sin = ang.cos().contiguous(), ang.sin().contiguous()
    y = torch.empty_like(x)
    ops.rope(x, y, 20, cos, sin, 10)
    xc = torch.view_as_complex(x.view(Bt, L, D // 2, 2))
    f = torch.polar(torch.ones_like(ang), ang).repeat(2, 1)
    ref = torch.view_as_real(xc * f).flatten(2)
    _close(y, ref, 1e-6)
    z = torch.empty_like(x)
    ops.rope(y, z, 20, cos, sin, 10, inverse=True)
    _close(z, x, 1e-6)


@pytest.mark.parametrize("dtype,D,nrot", [(torch.bfloat16, 256, 1024), (torch.float32, 64, 50), (torch.bfloat16, 6, 7)])
def test_rope_vector_path(dtype, D, nrot):
    """16-B vector RoPE (D % 8 == 0, aligned views) and the scalar fallback (D = 6) on strided
    views that rotate only the first nrot rows; inverse undoes it."""
    ops = _ops()
    torch.manual_seed(12)
    Bt, L = 3, nrot + 4
    base = torch.randn(Bt, L, D + 8, device=DEV).to(dtype)
    x = base[:, :, :D]
    ang = torch.rand(nrot // 2 + 1, D // 2, device=DEV) * 6
    cos, sin = ang.cos().contiguous(), ang.sin().contiguous()
    y = torch.zeros(Bt, L, D, device=DEV, dtype=dtype)
    ops.rope(x, y, nrot, cos, sin, nrot // 2 + 1)
    per = nrot // 2 + 1
    idx = torch.arange(nrot, device=DEV) % per
    xc = torch.view_as_complex(x[:, :nrot].float().reshape(Bt, nrot, D // 2, 2).contiguous())
    f = torch.polar(torch.ones_like(ang[idx]), ang[idx])
    ref = torch.view_as_real(xc * f).flatten(2)
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
    _close(y[:, :nrot], ref, tol)
    assert (y[:, nrot:] == 0).all()
    z = torch.zeros_like(y)
    ops.rope(y, z, nrot, cos, sin, per, inverse=True)
    _close(z[:, :nrot], x[:, :nrot].float(), 2 * tol)


@pytest.mark.parametrize("dtype,C,H,ws", [(torch.bfloat16, 112, 18, 8), (torch.float32, 96, 14, 7),
                                          (torch.bfloat16, 12, 9, 4)])
def test_window_partition_roundtrip(dtype, C, H, ws):
    """window partition (zero padding) / unpartition (padding dropped), plain and accumulating,
    vector (C % 8) and scalar (C = 12) paths against a torch reference"""
    ops = _ops()
    torch.manual_seed(13)
    B, W = 2, H + 3
    x = torch.randn(B, H, W, C, device=DEV).to(dtype)
    nh, nw = -(-H // ws), -(-W // ws)
    xp = torch.nn.functional.pad(x.float(), (0, 0, 0, nw * ws - W, 0, nh * ws - H))
    ref = xp.view(B, nh, ws, nw, ws, C).permute(0, 1, 3, 2, 4, 5).reshape(B * nh * nw, ws, ws, C)
    win = ops.window_partition(x, ws)
    _close(win, ref, 0)
    acc = torch.ones_like(win)
    ops.window_partition(x, ws, out=acc, accumulate=True)
    _close(acc, ref + 1, 1e-2 if dtype == torch.bfloat16 else 1e-6)
    back = ops.window_unpartition(win, ws, B, H, W)
    _close(back, x.float(), 0)
    acc2 = torch.ones_like(x)
    ops.window_unpartition(win, ws, B, H, W, out=acc2, accumulate=True)
    _close(acc2, x.float() + 1, 1e-2 if dtype == torch.bfloat16 else 1e-6)


@pytest.mark.parametrize("P", [4096, 4099])
def test_mask_loss_and_adamw(P):
    """P 4096: the 4-pixel vector kernels; 4099: the scalar fallback (P not a multiple of 4)"""
    ops = _ops()
    torch.manual_seed(3)
    N = 5
    x = torch.randn(N, P, device=DEV) * 3
    t = (torch.rand(N, P, device=DEV) > 0.7)
    t[2] = False
    stats = ops.mask_stats(x, t.view(torch.uint8))
    xs = x.clone().requires_grad_(True)
    tf = t.float()
    pr = xs.sigmoid()
    ce = torch.nn.functional.binary_cross_entropy_with_logits(xs, tf, reduction="none")
    p_t = pr * tf + (1 - pr) * (1 - tf)
    focal = (0.25 * tf + 0.75 * (1 - tf)) * ce * (1 - p_t) ** 2
    _close(stats[:, 0], focal.detach().sum(1), 1e-5)
    _close(stats[:, 1], pr.detach().sum(1), 1e-5)
    valid = t.any(1).int()
    pred_iou = torch.rand(N, device=DEV)
    losses = torch.zeros(4, device=DEV)
    coef = torch.empty(N, 4, device=DEV)
    ops.mask_loss_finalize(stats, pred_iou, valid, P, (20.0, 1.0, 1.0), 1.0, losses, coef)
    v = valid.bool()
    nv = v.sum()
    lm = (focal.mean(1)[v]).sum() / nv
    num = 2 * (pr * tf).sum(1) + 1
    den = pr.sum(1) + tf.sum(1) + 1
    ld = ((1 - num / den)[v]).sum() / nv
    tot = 20 * lm + ld
    _close(losses[0], lm.detach(), 1e-5)
    _close(losses[1], ld.detach(), 1e-5)
    tot.backward()
    dx = torch.empty_like(x)
    ops.mask_loss_bwd(x, t.view(torch.uint8), coef, 1.0, dx)
    _close(dx, xs.grad, 1e-4)
    # AdamW vs torch.optim.AdamW
    p = torch.randn(1000, device=DEV)
    g = torch.randn(1000, device=DEV)
    pt = p.clone().requires_grad_(True)
    opt = torch.optim.AdamW([pt], lr=1e-3, weight_decay=0.01, betas=(0.9, 0.999))
    m = torch.zeros_like(p)
    vv = torch.zeros_like(p)
    for step in range(1, 4):
        pt.grad = g.clone()
        opt.step()
        ops.adamw(p, g, m, vv, None, 1e-3, 0.9, 0.999, 1e-8, 0.01, step)
    _close(p, pt.detach(), 1e-6)


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-4), (torch.bfloat16, 2e-2)])
@pytest.mark.parametrize("cin,cout,H", [(1, 4, 37), (4, 16, 20), (16, 64, 15)])
def test_mask_down_stage(dtype, tol, cin, cout, H):
    """fused conv3x3/2 + LayerNorm2d + GELU (memory_encoder.py:17-55) vs torch fp32"""
    ops = _ops()
    O, W = 3, H + 3
    w = torch.randn(cout, cin, 3, 3, device=DEV) * 0.3
    b = torch.randn(cout, device=DEV) * 0.1
    g = torch.randn(cout, device=DEV)
    be = torch.randn(cout, device=DEV) * 0.1

    def ref(xin):
        y = _cpu_conv(torch.nn.functional.conv2d, xin.permute(0, 3, 1, 2), w, b, stride=2, padding=1)
        y = torch.nn.functional.layer_norm(y.permute(0, 2, 3, 1), (cout,), g, be, 1e-6)
        return torch.nn.functional.gelu(y)

    if cin == 1:
        logits = torch.randn(O, H, W, device=DEV) * 4
        y = ops.mask_down_stage(None, w, b, g, be, 1e-6, logits=logits, scale=20.0, shift=-10.0, dtype=dtype)
        xin = (torch.sigmoid(logits) * 20 - 10).to(dtype).float().unsqueeze(-1)
        _close(y, ref(xin), tol)
    x = torch.randn(O, H, W, cin, device=DEV).to(dtype)
    y = ops.mask_down_stage(x, w, b, g, be, 1e-6)
    _close(y, ref(x.float()), tol)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("act", [None, "relu", "gelu"])
def test_act_dropout_bwd_fused(dtype, act):
    """one-pass act' * dropout backward == dropout backward then act backward (same mask)"""
    ops = _ops()
    torch.manual_seed(3)
    pre = torch.randn(1000, 77, device=DEV).to(dtype)
    dy = torch.randn(1000, 77, device=DEV).to(dtype)
    got = ops.act_dropout_bwd(pre if act else None, dy, act, 0.1, 4321)
    g = ops.dropout(dy, 0.1, 4321)
    ref = ops.act_bwd(pre, g, act) if act else g
    _close(got, ref, 1e-2 if dtype == torch.bfloat16 else 1e-6)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_relu_mask_bwd_from_output(dtype, p):
    """ReLU -> dropout backward from the layer OUTPUT (s2h_relu_mask_bwd, and fused into the next
    layer's dgrad epilogue with alpha = 1/keep) == the pre-activation + re-hash backward
    (s2h_act_dropout_bwd) of the same linear epilogue"""
    ops = _ops()
    torch.manual_seed(5)
    M, K, N, N2 = 1000, 64, 136, 48
    x = torch.randn(M, K, device=DEV).to(dtype)
    w = (torch.randn(N, K, device=DEV) * 0.2).to(dtype)
    b = torch.randn(N, device=DEV) * 0.1
    pre = torch.empty(M, N, device=DEV, dtype=dtype)
    out = ops.linear(x, w, b, act="relu", pre=pre, drop_p=p, seed=99)
    dy = torch.randn(M, N, device=DEV).to(dtype)
    ref = ops.act_dropout_bwd(pre, dy, "relu", p, 99) if p > 0 else ops.act_bwd(pre, dy, "relu")
    got = ops.relu_mask_bwd(out, dy, 1.0 / (1.0 - p))
    _close(got, ref, 1e-6 if dtype == torch.float32 else 1e-2)
    # fused into the consumer's dgrad: dh = (dz @ w2) masked by out > 0, times 1/keep
    w2 = (torch.randn(N2, N, device=DEV) * 0.2).to(dtype)
    dz = torch.randn(M, N2, device=DEV).to(dtype)
    fused = ops.linear_dgrad(dz, w2, pre=out, act="relu", alpha=1.0 / (1.0 - p))
    plain = ops.relu_mask_bwd(out, ops.linear_dgrad(dz, w2), 1.0 / (1.0 - p))
    _close(fused, plain, 1e-5 if dtype == torch.float32 else 2e-2)


@pytest.mark.parametrize("max_norm,grad_scale", [(1.0, 1.0), (1.0, 0.5), (0.1, 0.25), (0.0, 0.5)])
def test_clip_adamw_matches_torch(max_norm, grad_scale):
    """s2h_grad_norm + s2h_adamw (ArenaAdamW) == clip_grad_norm_ + torch.optim.AdamW on the
    scaled gradient: grad_scale models the 1/world average after the SUM all-reduce (world 2 ->
    0.5) and 1/accumulate_grad_batches; max_norm 0 = no clip (Lightning's gradient_clip_val 0)"""
    ops = _ops()
    torch.manual_seed(11)
    n = 300_001
    p = torch.randn(n, device=DEV)
    pt = p.clone().requires_grad_(True)
    opt = torch.optim.AdamW([pt], lr=1e-3, weight_decay=0.01, betas=(0.9, 0.999))
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    ws, out = torch.empty(1024, device=DEV), torch.zeros(2, device=DEV)
    for step in range(1, 4):
        g = torch.randn(n, device=DEV) * (3.0 if step == 2 else 0.01)  # step 2 clips, the others do not
        pt.grad = g * grad_scale
        if max_norm > 0:
            torch.nn.utils.clip_grad_norm_([pt], max_norm)
        opt.step()
        ops.grad_norm(g, max_norm, ws, out, grad_scale)
        ops.adamw(p, g, m, v, out, 1e-3, 0.9, 0.999, 1e-8, 0.01, step)
        _close(out[0:1], (g * grad_scale).norm().view(1), 1e-5)
    _close(p, pt.detach(), 1e-5)


@pytest.mark.parametrize("N,hi,wi,ho,wo", [(104, 256, 256, 512, 512), (3, 64, 64, 256, 256), (2, 30, 17, 100, 61),
                                          (2, 64, 64, 32, 32)])
def test_bilinear_backward_matches_torch(N, hi, wi, ho, wo):
    """s2h_bilinear_bwd (the gather form with the column taps hoisted, round 6) against torch's
    upsample_bilinear2d backward (align_corners=False): the step's 104-plane 256^2 -> 512^2 mask
    upsampling, 4x, a non-integer ratio and a down-sampling"""
    ops = _ops()
    torch.manual_seed(13)
    x = torch.randn(N, hi, wi, device=DEV, requires_grad=True)
    g = torch.randn(N, ho, wo, device=DEV)
    torch.nn.functional.interpolate(x[:, None], size=(ho, wo), mode="bilinear", align_corners=False)[:, 0].backward(g)
    _close(ops.bilinear_bwd(g, hi, wi), x.grad, 1e-5)


@pytest.mark.parametrize("out_dtype,alpha", [(torch.bfloat16, 1.0), (torch.float32, 0.5)])
def test_k1_outer_product_path_equals_tiled_gemm(out_dtype, alpha):
    """K = 1 GEMMs (the hypernetwork-mask gradient dup[o] = g[o]^T h[o], 104 x 16384 x 32) take the
    element-wise outer-product kernel (round 6): the same bits as the tiled MFMA GEMM (forced with
    s2h_gemm_config), batched with strides, N not a multiple of 8 included"""
    from sam2_video.kernels import _lib
    ops = _ops()
    torch.manual_seed(14)
    for Bt, M, N in ((104, 16384, 32), (3, 100, 37)):
        g = torch.randn(Bt, 1, M, device=DEV).to(torch.bfloat16)
        h = torch.randn(Bt, 1, N, device=DEV).to(torch.bfloat16)
        outs = []
        for cfg in (0, 1):  # 0: the shape rules (outer-product path), 1: the 64 x 64 tiling
            prev = _lib.lib().s2h_gemm_config(cfg)
            try:
                out = torch.full((Bt, M, N), float("nan"), device=DEV, dtype=out_dtype)
                ops.gemm(g, h, out, M=M, N=N, K=1, lda_m=1, lda_k=M, ldb_k=N, ldb_n=1, ldc=N, batch=Bt, sA=M, sB=N,
                         sC=M * N, alpha=alpha)
                torch.cuda.synchronize()
                outs.append(out)
            finally:
                _lib.lib().s2h_gemm_config(prev)
        assert torch.equal(outs[0], outs[1])
        ref = alpha * g.float().transpose(1, 2) @ h.float()
        _close(outs[0].float(), ref, 1e-2)


@pytest.mark.parametrize("M,N,K", [(256, 256, 72), (256, 72, 256), (100, 37, 130)])
def test_small_fp32_gemm_tilings(M, N, K):
    """fp32 GEMMs of fewer than 64 tiles of 64^2 (the V-fold weight gradients) on 32 x 32 tiles (round 6,
    s2h_gemm_f32_small(1)) and on 64 x 64: both against the fp64 product, NN / TN layouts, beta 1"""
    from sam2_video.kernels._lib import lib
    ops = _ops()
    torch.manual_seed(17)
    a = torch.randn(M, K, device=DEV)
    at = a.t().contiguous()  # [K, M]: A with m contiguous
    b = torch.randn(K, N, device=DEV)
    c0 = torch.randn(M, N, device=DEV)
    ref = a.double() @ b.double()
    prev = lib().s2h_gemm_f32_small(-1)
    try:
        for mode in (1, 0):
            lib().s2h_gemm_f32_small(mode)
            c = torch.empty(M, N, device=DEV)
            ops.gemm(a, b, c, M=M, N=N, K=K, lda_m=K, lda_k=1, ldb_k=N, ldb_n=1, ldc=N)
            _close(c, ref.float(), 1e-5)
            c = c0.clone()
            ops.gemm(at, b, c, M=M, N=N, K=K, lda_m=1, lda_k=M, ldb_k=N, ldb_n=1, ldc=N, beta=1.0)
            _close(c, (ref + c0.double()).float(), 1e-5)
    finally:
        lib().s2h_gemm_f32_small(prev)


def test_adamw_vector_and_scalar_paths_bit_identical():
    """s2h_adamw's 16-B-per-lane kernel (aligned arena, the step's case) and its scalar form (unaligned
    pointers, and the n % 4 tail) compute the same update element for element, bf16 shadow included"""
    ops = _ops()
    torch.manual_seed(12)
    n = 100_003
    src = [torch.randn(n, device=DEV) for _ in range(4)]
    src[3] = src[3].abs()  # v >= 0
    clip = torch.tensor([0.0, 0.7], device=DEV)
    out = []
    for off in (0, 1):  # 0: 16-B aligned (vector kernel + 3-element tail), 1: 4-B offset (scalar kernel)
        p, g, m, v = (torch.empty(n + 1, device=DEV)[off:off + n].copy_(t) for t in src)
        sh = torch.empty(n + 4, device=DEV, dtype=torch.bfloat16)[4 * off:4 * off + n]
        for step in (1, 2):
            ops.adamw(p, g, m, v, clip, 1e-3, 0.9, 0.999, 1e-8, 0.01, step, shadow=sh)
        torch.cuda.synchronize()
        out.append((p, m, v, sh))
    for a, b in zip(*out):
        assert torch.equal(a, b)


def test_category_merge_multi_object_matches_reference_formulas():
    """merge_masks / merge_scores over categories of 1, 2 and 3 objects (a tie and a NaN included)
    vs the reference's _grouped_max / _grouped_weighted_avg (masks.py:92-143) under autograd:
    forward values and the gradients into the object logits and scores"""
    from sam2_video.utils.masks import merge_object_results_to_category
    torch.manual_seed(5)
    obj_to_cat = [0, 1, 1, 2, 2, 2]
    O, H = len(obj_to_cat), 24
    logits = torch.randn(O, 1, H, H, device=DEV) * 3
    logits[2, 0, 0, 0] = logits[1, 0, 0, 0]  # exact tie: the first object takes the gradient
    ious = torch.rand(O, 1, device=DEV)
    stage = {"pred_masks": logits, "pred_masks_high_res": logits, "multistep_pred_masks": logits,
             "multistep_pred_masks_high_res": logits, "multistep_pred_multimasks": [logits],
             "multistep_pred_multimasks_high_res": [logits], "multistep_pred_ious": [ious],
             "multistep_object_score_logits": [ious], "point_inputs": None, "mask_inputs": None}
    x = logits.clone().requires_grad_(True)
    s = ious.clone().requires_grad_(True)
    st = dict(stage, pred_masks_high_res=x, multistep_pred_multimasks_high_res=[x], multistep_pred_ious=[s])
    out = merge_object_results_to_category([st], obj_to_cat, 3)[0]
    hr, mi = out["multistep_pred_multimasks_high_res"][0], out["multistep_pred_ious"][0]
    # reference formulas on the same inputs
    xr = logits.clone().requires_grad_(True)
    sr = ious.clone().requires_grad_(True)
    groups = [[0], [1, 2], [3, 4, 5]]
    w = torch.sigmoid(xr).sum(dim=(1, 2, 3))
    hr_ref = torch.stack([xr[g].max(dim=0).values for g in groups])
    mi_ref = torch.stack([(sr[g] * w[g].view(-1, 1)).sum(0) / w[g].sum() for g in groups])
    _close(hr, hr_ref, 1e-6)
    _close(mi, mi_ref, 1e-5)
    gh = torch.randn_like(hr_ref)
    gi = torch.randn_like(mi_ref)
    ((hr * gh).sum() + (mi * gi).sum()).backward()
    ((hr_ref * gh).sum() + (mi_ref * gi).sum()).backward()
    _close(x.grad, xr.grad, 1e-4)
    _close(s.grad, sr.grad, 1e-5)
    # the one-node merge (merge_masks_scores) gives the bits of the two separate nodes
    from sam2_video.kernels.functional_sam import merge_scores
    from sam2_video.utils.masks import CategoryGroups as _CG
    x2 = logits.clone().requires_grad_(True)
    s2 = ious.clone().requires_grad_(True)
    grp = _CG(obj_to_cat, 3, x2.device)
    from sam2_video.kernels.functional_sam import merge_masks as _mm
    ((_mm(x2, grp) * gh).sum() + (merge_scores(s2, x2, grp) * gi).sum()).backward()
    assert torch.equal(x.grad, x2.grad) and torch.equal(s.grad, s2.grad)
    # the object-score merge reuses the high-res statistics of that node: the bits of merge_scores
    with torch.no_grad():
        assert torch.equal(out["multistep_object_score_logits"][0], merge_scores(ious, logits, grp))
    # a NaN logit propagates through the max like torch.max (the kernel once dropped it)
    from sam2_video.kernels.functional_sam import merge_masks
    from sam2_video.utils.masks import CategoryGroups
    xn = logits.clone()
    xn[4, 0, 1, 1] = float("nan")
    got = merge_masks(xn, CategoryGroups(obj_to_cat, 3, xn.device))
    ref = torch.stack([xn[g].max(dim=0).values for g in groups])
    assert torch.equal(torch.isnan(got), torch.isnan(ref)) and bool(torch.isnan(got[2, 0, 1, 1]))


@pytest.mark.parametrize("reduction,pw,temp", [("mean", None, 1.0), ("mean", [0.5, 2.0, 1.0, 3.0], 0.7),
                                               ("sum", None, 1.5)])
def test_bce_category_loss_matches_reference_formula(reduction, pw, temp):
    """BCECategoryLoss (losses.py:251-372) vs its torch formula: valid-category filter, logit
    temperature, pos_weight, mean/sum reduction, average over frames; loss and d(logits)"""
    import torch.nn.functional as F

    from sam2_video.model.losses import BCECategoryLoss
    torch.manual_seed(8)
    T, C, H = 3, 4, 40
    logits = torch.randn(T, C, 1, H, H, device=DEV) * 2
    tgt = torch.rand(T, C, H, H, device=DEV) > 0.6
    tgt[1, 2] = False  # a category without ground truth in frame 1
    x = logits.clone().requires_grad_(True)
    outs = [{"pred_masks_high_res": x[t]} for t in range(T)]
    crit = BCECategoryLoss(pos_weight=pw, reduction=reduction, logit_temperature=temp)
    got = crit(outs, tgt)
    xr = logits.clone().requires_grad_(True)
    tot = 0.0
    for t in range(T):
        valid = tgt[t].sum(dim=(1, 2)).bool()
        lw = None if pw is None else torch.tensor(pw, device=DEV).view(-1, 1, 1)[valid]
        tot = tot + F.binary_cross_entropy_with_logits(xr[t].squeeze(1)[valid] / temp, tgt[t][valid].float(),
                                                       pos_weight=lw, reduction=reduction)
    tot = tot / T
    _close(got["total_loss"].view(1), tot.view(1), 1e-5)
    assert torch.equal(got["loss_bce"], got["total_loss"])
    got["total_loss"].backward()
    tot.backward()
    _close(x.grad, xr.grad, 1e-5)


@pytest.mark.parametrize("d", [56, 72])
def test_flash_strided_qkv_padded_head_fwd_bwd(d):
    """Hiera's fused [B, L, 3, H, d] projection (B+ 56, L 72) through the padded 64 / 128 flash
    path: q / k / v read in place, gradients written in place into one dqkv buffer (the QKV
    attention layout)"""
    ops = _ops()
    torch.manual_seed(8)
    B, L, H = 3, 196, 2
    qkv = (torch.randn(B, L, 3, H, d, device=DEV) * 0.7).to(torch.bfloat16)
    q, k, v = qkv.unbind(2)
    o = torch.empty(B, L, H, d, device=DEV, dtype=torch.bfloat16)
    lse = torch.empty(B, H, L, device=DEV)
    ops.attn_fwd(q, k, v, o, lse, d ** -0.5)
    qr, kr, vr = (t.float().clone().requires_grad_(True) for t in (q, k, v))
    ro, rl = _ref_attn(qr, kr, vr, d ** -0.5)
    _close(o, ro, 2e-2)
    _close(lse, rl, 1e-3)
    do = torch.randn_like(o)
    ro.backward(do.float())
    dqkv = torch.full((B, L, 3, H, d), float("nan"), device=DEV, dtype=torch.bfloat16)
    dq, dk, dv = dqkv.unbind(2)
    ops.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, d ** -0.5)
    _close(dq, qr.grad, 4e-2)
    _close(dk, kr.grad, 4e-2)
    _close(dv, vr.grad, 4e-2)


def test_flash_bwd_strided_o_and_misaligned_o_refused():
    """the flash dQ kernel reads O (Di fusion) with 16-B loads: O as a strided view into a wider
    buffer (16-B aligned base and strides) gives the contiguous-O gradients bit for bit; an O whose
    base is only 8-B aligned goes to the generic kernel through s2h_attn_bwd, and is refused with
    hipErrorInvalidValue by the frame-batched flash entry point instead of faulting"""
    ops = _ops()
    from sam2_video.kernels._lib import HipKernelError
    torch.manual_seed(9)
    B, L, H, D = 2, 256, 1, 256
    q, k, v = ((torch.randn(B, L, H, D, device=DEV) * 0.5).to(torch.bfloat16) for _ in range(3))
    o = torch.empty(B, L, H, D, device=DEV, dtype=torch.bfloat16)
    lse = torch.empty(B, H, L, device=DEV)
    ops.attn_fwd(q, k, v, o, lse, D ** -0.5)
    do = torch.randn_like(o)
    grads = [torch.empty_like(q) for _ in range(3)]
    ops.attn_bwd(q, k, v, o, do, lse, *grads, D ** -0.5)
    wide = torch.zeros(B, L, H, D + 16, device=DEV, dtype=torch.bfloat16)
    ow = wide[..., 8:8 + D]
    ow.copy_(o)
    g2 = [torch.empty_like(q) for _ in range(3)]
    ops.attn_bwd(q, k, v, ow, do, lse, *g2, D ** -0.5)
    for a, b in zip(grads, g2):
        assert torch.equal(a, b)
    om = wide[..., 4:4 + D]
    om.copy_(o)
    g3 = [torch.empty_like(q) for _ in range(3)]
    ops.attn_bwd(q, k, v, om, do, lse, *g3, D ** -0.5)  # generic kernel
    for a, b in zip(grads, g3):
        _close(b, a.float(), 4e-2)
    kp, vp = k.reshape(B * L, H, D), v.reshape(B * L, H, D)
    with pytest.raises(HipKernelError):
        ops.flash_bwd_frames(1, B, [L], [0], [0], q, kp, vp, om, do, lse, torch.empty_like(q),
                             torch.empty_like(kp), torch.empty_like(vp), D ** -0.5, 0.0, 0)
    torch.cuda.synchronize()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_elementwise_vector_forms_match_scalar(dtype):
    """16-B vector kernels (add, broadcast add, act fwd / bwd, dropout, act + dropout backward)
    give bit-identical results to the scalar kernels (selected by 2-byte-misaligned views) and
    match torch on the plain ops; odd dropout index offsets take the per-element hash path"""
    ops = _ops()
    torch.manual_seed(11)
    R, C = 999, 264
    n = R * C

    def pair():  # the same values aligned (vector path) and misaligned (scalar path)
        buf = torch.randn(n + 1, device=DEV).to(dtype)
        al = torch.empty(n, device=DEV, dtype=dtype)
        al.copy_(buf[1:])
        return al, buf[1:]

    (a, a_), (b, b_) = pair(), pair()
    assert a.data_ptr() % 16 == 0 and a_.data_ptr() % 16 != 0
    out_ = torch.empty(n + 1, device=DEV, dtype=dtype)[1:]
    for alpha, beta in ((1.0, 1.0), (0.5, -2.0)):
        v = ops.add(a, b, alpha=alpha, beta=beta)
        s = ops.add(a_, b_, out=out_, alpha=alpha, beta=beta)
        assert torch.equal(v, s)
        _close(v, (alpha * a.float() + beta * b.float()).to(dtype), 1e-2 if dtype == torch.bfloat16 else 1e-6)
    tab, tab_ = pair()
    for period in (1, 7):
        v = ops.add_bcast(a.view(R, C), tab[: period * C], b_period=period, alpha=0.7, beta=1.3)
        s = ops.add_bcast(a_.view(R, C), tab_[: period * C], out=out_.view(R, C), b_period=period, alpha=0.7, beta=1.3)
        assert torch.equal(v.reshape(-1), s.reshape(-1)), period
        ref = 0.7 * a.float().view(R, C) + 1.3 * tab[: period * C].float().view(period, C).repeat(R // period + 1, 1)[:R]
        _close(v.view(R, C), ref.to(dtype), 2e-2 if dtype == torch.bfloat16 else 1e-5)
    for act in ("relu", "gelu"):
        assert torch.equal(ops.act_fwd(a, act), ops.act_fwd(a_, act, out=out_))
        assert torch.equal(ops.act_bwd(a, b, act), ops.act_bwd(a_, b_, act, dx=out_))
    for idx0 in (0, 3):
        assert torch.equal(ops.dropout(b, 0.1, 77, idx0=idx0), ops.dropout(b_, 0.1, 77, out=out_, idx0=idx0))
        assert torch.equal(ops.act_dropout_bwd(a, b, "gelu", 0.1, 77, idx0=idx0),
                           ops.act_dropout_bwd(a_, b_, "gelu", 0.1, 77, dx=out_, idx0=idx0))



@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("Bt,L,nrot,N,ncol,dh", [(3, 256, 256, 256, 256, 256), (2, 1028 + 8, 1028, 256, 256, 256),
                                                  (2, 256, 256, 768, 512, 256), (4, 64, 48, 128, 128, 32)])
def test_linear_rope_matches_linear_then_rope(dtype, Bt, L, nrot, N, ncol, dh):
    """s2h_linear_rope (RoPE in the GEMM epilogue: q / k projections, the fused q/k/v projection
    with q and k rotated, key rows past nrot -- object-pointer tokens -- left alone) against the
    torch fp32 product followed by the reference's complex-pair rotation (position_encoding.py:
    212-239, table row r % period); and rope_blocks(inverse) undoes it"""
    ops = _ops()
    from sam2_video.model.modeling.position_encoding import axial_rope_table
    torch.manual_seed(3)
    period = 64 if dh == 32 else 256
    side = int(period ** 0.5)
    cos, sin = axial_rope_table(dh, side, side, 10000.0, DEV)
    K = 64 if N == 256 and L > 1000 else 256
    x = (torch.randn(Bt, L, K, device=DEV) * 0.5).to(dtype)
    w = (torch.randn(N, K, device=DEV) * 0.05).to(dtype)
    b = torch.randn(N, device=DEV)
    y = ops.linear_rope(x, w, b, (cos, sin, L, nrot, period, ncol, dh))
    ref = (x.float() @ w.float().t() + b).view(Bt, L, N).clone()
    cc = torch.complex(cos, sin)  # [period, dh / 2]
    for c0 in range(0, ncol, dh):
        blk = ref[:, :nrot, c0:c0 + dh].reshape(Bt, nrot, dh // 2, 2)
        z = torch.view_as_complex(blk.contiguous()) * cc[torch.arange(nrot, device=DEV) % period]
        ref[:, :nrot, c0:c0 + dh] = torch.view_as_real(z).reshape(Bt, nrot, dh)
    _close(y, ref, 2e-2 if dtype == torch.bfloat16 else 1e-5)
    back = y.clone().view(-1, N)
    ops.rope_blocks(back, (cos, sin, L, nrot, period, ncol, dh), inverse=True)
    _close(back.view(Bt, L, N), (x.float() @ w.float().t() + b), 3e-2 if dtype == torch.bfloat16 else 1e-5)


@pytest.mark.parametrize("M,N,K", [(13312, 256, 256), (13312, 256, 72), (13312, 256, 2048), (1000, 256, 200),
                                   (13312, 128, 256), (333, 128, 64)])
@pytest.mark.parametrize("p_drop,res", [(0.0, True), (0.1, True), (0.1, False)])
def test_linear_add_ln_matches_unfused(M, N, K, p_drop, res):
    """s2h_linear_add_ln (projection + dropout + residual + LayerNorm in one full-row launch) against
    the unfused pair ops.linear(..., residual, dropout) + ops.layernorm_fwd: the residual stream x'
    bit-identical (same tiling order over K, same epilogue), LN(x') / mean / rstd within fp32
    summation order (one bf16 rounding of y)"""
    ops = _ops()
    torch.manual_seed(5)
    bf = torch.bfloat16
    ops.rng_offset(DEV).fill_(7)
    x = torch.randn(M, K, device=DEV).to(bf)
    w = (torch.randn(N, K, device=DEV) / K ** 0.5).to(bf)
    b = torch.randn(N, device=DEV) * 0.1
    r = torch.randn(M, N, device=DEV).to(bf) if res else None
    g = torch.rand(N, device=DEV) + 0.5
    be = torch.randn(N, device=DEV) * 0.1
    y, xs, mean, rstd = ops.linear_add_ln(x, w, b, r, g, be, 1e-5, drop_p=p_drop, seed=99, drop_idx0=12)
    ref_x = ops.linear(x, w, b, residual=r, drop_p=p_drop, seed=99, drop_idx0=12)
    assert torch.equal(xs, ref_x)
    ref_y, ref_m, ref_r = ops.layernorm_fwd(ref_x, g, be, 1e-5)
    _close(y, ref_y, 8e-3)
    torch.testing.assert_close(mean, ref_m, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(rstd, ref_r, atol=1e-5, rtol=1e-4)
    # and against fp32 torch (LayerNorm of the bf16 residual stream)
    t = torch.nn.functional.layer_norm(ref_x.float(), (N,), g, be, 1e-5)
    _close(y, t, 8e-3)


@pytest.mark.parametrize("M,C,K", [(13312, 256, 768), (13312, 256, 256), (93184, 256, 2048), (1000, 256, 200),
                                   (13312, 128, 256), (333, 128, 64)])
@pytest.mark.parametrize("res,wgrad", [(True, True), (False, True), (True, False)])
def test_linear_dgrad_ln_bwd_matches_unfused(M, C, K, res, wgrad):
    """s2h_linear_dgrad_ln_bwd (a Linear's input gradient with the backward of the LayerNorm that
    produced its input in the GEMM epilogue) against the unfused pair ops.linear_dgrad ->
    ops.layernorm_bwd and against fp32 torch autograd of layer_norm -> linear: the fused path keeps
    dL/dt in fp32 (the unfused one rounds it to bf16 once), so dx agrees within bf16 rounding and the
    LayerNorm weight gradients within fp32 summation order"""
    ops = _ops()
    torch.manual_seed(11)
    bf = torch.bfloat16
    x = (torch.randn(M, C, device=DEV) * 2 + 0.3).to(bf)
    g = torch.rand(C, device=DEV) + 0.5
    be = torch.randn(C, device=DEV) * 0.1
    w = (torch.randn(K, C, device=DEV) / C ** 0.5).to(bf)  # the consumer Linear: C -> K
    dy = torch.randn(M, K, device=DEV).to(bf)
    dres = torch.randn(M, C, device=DEV).to(bf) if res else None
    _, mean, rstd = ops.layernorm_fwd(x, g, be, 1e-5)
    dg = torch.zeros(C, device=DEV) if wgrad else None
    db = torch.zeros(C, device=DEV) if wgrad else None
    dx = ops.linear_dgrad_ln_bwd(dy, w, x, g, mean, rstd, dres=dres, dgamma=dg, dbeta=db)
    # unfused twin
    dt = ops.linear_dgrad(dy, w)
    dg2 = torch.zeros(C, device=DEV) if wgrad else None
    db2 = torch.zeros(C, device=DEV) if wgrad else None
    dx2 = ops.layernorm_bwd(x, dt, g, mean, rstd, dgamma=dg2, dbeta=db2,
                            dres=dres.contiguous() if dres is not None else None)
    _close(dx, dx2, 1.5e-2)
    # fp32 torch reference of the same composition
    xr = x.float().requires_grad_(True)
    gr = g.clone().requires_grad_(True)
    br = be.clone().requires_grad_(True)
    t = torch.nn.functional.layer_norm(xr, (C,), gr, br, 1e-5)
    (t @ w.float().t()).backward(dy.float())
    ref = xr.grad + (dres.float() if dres is not None else 0)
    _close(dx, ref, 1e-2)
    if wgrad:
        _close(dg, gr.grad, 2e-3)
        _close(db, br.grad, 2e-3)
        _close(dg, dg2, 1e-2)
        _close(db, db2, 1e-2)


@pytest.mark.parametrize("cfg", [29, 30])
@pytest.mark.parametrize("M,N,K,bkc", [(13312, 256, 256, True), (13312, 768, 256, True), (93184, 256, 256, False),
                                       (1000, 200, 136, True), (70, 24, 40, False), (13312, 2048, 256, False)])
def test_areg_tiling_bit_identical(cfg, M, N, K, bkc):
    """the short-K tilings with A in registers (gemm16a_kernel) accumulate every output over the same
    K order as the LDS-staged 64 x 64 tile, so with the same epilogue (bias, ReLU, dropout, residual)
    the results are bit-identical"""
    from sam2_video.kernels import _lib
    ops = _ops()
    torch.manual_seed(3)
    bf = torch.bfloat16
    ops.rng_offset(DEV).fill_(5)
    a = torch.randn(M, K, device=DEV).to(bf)
    b = torch.randn(N, K, device=DEV).to(bf) if bkc else torch.randn(K, N, device=DEV).to(bf)
    kw = dict(M=M, N=N, K=K, lda_m=K, lda_k=1, ldb_k=1 if bkc else N, ldb_n=K if bkc else 1, ldc=N)
    bias = torch.randn(N, device=DEV)
    res = torch.randn(M, N, device=DEV).to(bf)
    outs = []
    for c in (1, cfg):
        prev = _lib.lib().s2h_gemm_config(c)
        try:
            out = torch.empty(M, N, device=DEV, dtype=bf)
            ops.gemm(a, b, out, bias=bias, residual=res, ldr=N, act=1, drop_p=0.1, seed=17, **kw)
            outs.append(out)
        finally:
            _lib.lib().s2h_gemm_config(prev)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("M", [13, 3, 40])
def test_mlp_heads_bit_identical(M):
    """s2h_mlp_heads (no-grad per-object MLP heads in one launch: the object-score head and the
    object-pointer projection) against the per-layer GEMMs: same K order and epilogue arithmetic per
    layer, so bit-identical -- a strided input view (the decoder's token rows), 1- / 32- / 256-wide
    outputs, a sigmoid last layer, rows spanning several workgroups"""
    ops = _ops()
    torch.manual_seed(9)
    bf = torch.bfloat16
    hs = torch.randn(M, 9, 256, device=DEV).to(bf)
    specs = [(hs[:, 0], [256, 256, 256, 1], None), (hs[:, 2].contiguous(), [256, 256, 256, 256], None),
             (hs[:, 3].contiguous(), [256, 256, 256, 32], "sigmoid"), (hs[:, 1].contiguous(), [256, 128, 4], None)]
    heads, refs, rhid, rpre, hid, pre = [], [], [], [], [], []
    for x, dims, last_act in specs:
        ws = [(torch.randn(dims[i + 1], dims[i], device=DEV) / dims[i] ** 0.5).to(bf) for i in range(len(dims) - 1)]
        bs = [torch.randn(dims[i + 1], device=DEV) * 0.1 for i in range(len(dims) - 1)]
        heads.append((x, ws, bs, last_act))
        y = x.contiguous()
        hl = []
        for i, (w, b) in enumerate(zip(ws, bs)):
            last = i == len(ws) - 1
            p = torch.empty(M, w.shape[0], device=DEV, dtype=bf) if last and last_act else None
            y = ops.linear(y, w, b, act=("relu" if not last else last_act), pre=p)
            if not last:
                hl.append(y)
        refs.append(y)
        rhid.append(hl)
        rpre.append(p)
        hid.append([torch.empty_like(h) for h in hl])
        pre.append(torch.empty_like(p) if p is not None else None)
    outs = ops.mlp_heads(heads)
    for o, r in zip(outs, refs):
        assert torch.equal(o, r), float((o.float() - r.float()).abs().max())
    # with the saved hidden activations / last pre-activation (the trained heads' tape op)
    outs = ops.mlp_heads(heads, hidden=hid, pre=pre)
    for o, r, h, rh, p, rp in zip(outs, refs, hid, rhid, pre, rpre):
        assert torch.equal(o, r)
        for a, b in zip(h, rh):
            assert torch.equal(a, b)
        if rp is not None:
            assert torch.equal(p, rp)


@pytest.mark.parametrize("M,N,K", [(104, 256, 2048), (13, 256, 1024), (128, 64, 4096), (100, 250, 2048)])
def test_tiny_m_splitk_gemm_matches_one_launch_tiling(M, N, K):
    """round 6: bf16-output GEMMs with M <= 128 and K >= 1024 run as a split-K fp32 launch + a fixed-order
    reduce that applies the GEMM epilogue (gemm_bf16.hip gemm_tiny_splitk); against the one-launch tiling
    (s2h_gemm_tiny_splitk(0)) and the fp32 torch reference, with bias + GELU (+ pre-activation store),
    dropout and residual; bit-identical on repeat"""
    ops = _ops()
    from sam2_video.kernels._lib import lib
    torch.manual_seed(11)
    bf = torch.bfloat16
    x = torch.randn(M, K, device=DEV).to(bf)
    w = (torch.randn(N, K, device=DEV) * K ** -0.5).to(bf)
    b = torch.randn(N, device=DEV)
    r = torch.randn(M, N, device=DEV).to(bf)
    ref = x.float() @ w.float().t() + b
    outs = {}
    for mode in (1, 0, 1):  # (the split path is opt-in: forced on / off here)
        prev = lib().s2h_gemm_tiny_splitk(mode)
        try:
            pre = torch.empty(M, N, device=DEV, dtype=bf)
            y = ops.linear(x, w, b, act="gelu", pre=pre)
            yd = ops.linear(x, w, b, residual=r, drop_p=0.1, seed=5)
        finally:
            lib().s2h_gemm_tiny_splitk(prev)
        torch.cuda.synchronize()
        if mode in outs:
            assert all(torch.equal(u, v) for u, v in zip(outs[mode], (y, pre, yd)))
        outs[mode] = (y, pre, yd)
    y, pre, yd = outs[1]
    _close(pre, ref, 1e-2)
    _close(y, torch.nn.functional.gelu(ref), 1e-2)
    keep = outs[0][2] != r  # the one-launch tiling's dropout mask (same seed and element indices)
    _close(yd.float(), torch.where(keep, ref / 0.9 + r.float(), r.float()), 2e-2)
    for u, v in zip(outs[1], outs[0]):
        _close(u, v, 1e-2)
