"""Small backward reductions rewritten for parallelism in round 5 against torch references: the
bilinear upsampling gather (tight source window), the windowed positional-embedding gradient (16
slices + fixed tree), the point-label embedding gradient (register sums in row order)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.mark.parametrize("N,hi,wi,ho,wo", [(104, 128, 128, 512, 512), (3, 7, 9, 30, 17), (2, 40, 40, 13, 11)])
def test_bilinear_bwd_matches_autograd(N, hi, wi, ho, wo):
    from sam2_video.kernels import ops
    torch.manual_seed(0)
    x = torch.randn(N, hi, wi, device=DEV, requires_grad=True)
    y = torch.nn.functional.interpolate(x.unsqueeze(1), size=(ho, wo), mode="bilinear", align_corners=False)
    g = torch.randn_like(y)
    y.backward(g)
    dx = ops.bilinear_bwd(g.squeeze(1).contiguous(), hi, wi)
    torch.cuda.synchronize()
    assert (dx - x.grad).abs().max().item() <= 1e-5 * x.grad.abs().max().item()
    assert torch.equal(dx, ops.bilinear_bwd(g.squeeze(1).contiguous(), hi, wi))


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("h,w,C,ws", [(128, 128, 112, 8), (96, 80, 64, 8), (20, 12, 16, 7)])
def test_pos_window_grad(dtype, h, w, C, ws):
    from sam2_video.kernels import ops
    torch.manual_seed(1)
    dout = torch.randn(h, w, C, device=DEV).to(dtype)
    dwin = torch.full((C, ws, ws), 0.25, device=DEV)
    ops.pos_embed_bwd(dout, None, dwin, ws)
    ref = torch.full((C, ws, ws), 0.25, device=DEV, dtype=torch.float64)
    d = dout.double()
    for a in range(ws):
        for b in range(ws):
            ref[:, a, b] += d[a::ws, b::ws].sum((0, 1))
    torch.cuda.synchronize()
    assert (dwin.double() - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_point_embed_grad(dtype):
    from sam2_video.kernels import ops
    torch.manual_seed(2)
    R, D = 211, 256
    labels = torch.randint(-1, 4, (R,), device=DEV, dtype=torch.int32)
    dout = torch.randn(R, D, device=DEV).to(dtype)
    dtable = torch.randn(5, D, device=DEV)
    ref = dtable.clone()
    ops.point_embed_bwd(labels, dout, dtable)
    for r in range(R):  # the same additions in the same order
        ref[int(labels[r]) + 1] += dout[r].float()
    torch.cuda.synchronize()
    assert torch.equal(dtable, ref)


@pytest.mark.parametrize("dtype,F,O,inner", [(torch.bfloat16, 7, 13, 262144), (torch.float32, 3, 5, 1000),
                                             (torch.bfloat16, 2, 3, 50)])
def test_sum_outer_batched_equals_per_frame(dtype, F, O, inner):
    """the frame-batched broadcast-gradient sum (one launch) gives the bits of one sum_outer per frame"""
    from sam2_video.kernels import ops
    torch.manual_seed(3)
    x = torch.randn(F, O, inner, device=DEV).to(dtype)
    out = torch.empty(F * inner, device=DEV, dtype=dtype)
    ops.sum_outer_batched(x, out)
    ref = torch.empty_like(out)
    for f in range(F):
        ops.sum_outer(x[f], ref[f * inner:(f + 1) * inner])
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    t = x.double().sum(1).flatten()
    assert (out.double() - t).abs().max().item() <= (1e-2 if dtype == torch.bfloat16 else 1e-5) * t.abs().max().item()


def test_memory_encoder_pixel_add_in_projection_epilogue(monkeypatch):
    """the memory encoder's pix_feat_proj(pix_feat) + masks (memory_encoder.py:174-175) added in the
    mask down-sampler's final projection (one batched GEMM, residual with object stride 0) against the
    projection + broadcast add (S2H_MEMENC_ADD=0): equal to one bf16 rounding of the same fp32 sum"""
    import sys
    import os
    sys.path.insert(0, os.path.dirname(__file__))
    from step_harness import build_model
    model = build_model("base_plus", 256, ["memory_encoder"], dtype="bf16")
    enc = model.memory_encoder
    torch.manual_seed(6)
    h = w = 16
    pix = torch.randn(h * w, 256, device=DEV).to(torch.bfloat16)
    masks = torch.randn(13, 16 * h, 16 * w, device=DEV) * 4
    out = {}
    for flag in ("0", "1"):
        monkeypatch.setenv("S2H_MEMENC_ADD", flag)
        feat, pos = enc(pix, masks, h, w, scale=20.0, shift=-10.0)
        torch.cuda.synchronize()
        out[flag] = feat.float()
    a, b = out["1"], out["0"]
    assert torch.isfinite(a).all()
    # one bf16 rounding of x, carried through the fuser's CX blocks and the output projection
    assert (a - b).abs().max().item() <= 2e-2 * b.abs().max().item()
    assert torch.nn.functional.cosine_similarity(a.flatten().double(), b.flatten().double(), dim=0).item() >= 0.9999


@pytest.mark.parametrize("rows,L", [(13 * 1024, 1024), (3 * 64, 64), (40, 8)])
def test_layernorm_fwd_pe_equals_ln_then_add_bcast(rows, L):
    """s2h_layernorm_fwd_pe (norm4 + the next block's keys + key_pe, transformer.py:182-185, :170) gives
    the bits of the LayerNorm launch followed by the broadcast add"""
    from sam2_video.kernels import ops
    from sam2_video.kernels._lib import call
    torch.manual_seed(7)
    C = 256
    x = torch.randn(rows, C, device=DEV).to(torch.bfloat16)
    pe = torch.randn(L, C, device=DEV).to(torch.bfloat16)
    g = torch.randn(C, device=DEV)
    b = torch.randn(C, device=DEV)
    y = torch.empty_like(x)
    k = torch.empty_like(x)
    mean = torch.empty(rows, device=DEV)
    rstd = torch.empty(rows, device=DEV)
    call("s2h_layernorm_fwd_pe", 1, rows, C, x.data_ptr(), g.data_ptr(), b.data_ptr(), 1e-5, y.data_ptr(),
         mean.data_ptr(), rstd.data_ptr(), pe.data_ptr(), L, k.data_ptr(), ops.stream())
    ry, rm, rr = ops.layernorm_fwd(x, g, b, 1e-5)
    rk = ops.add_bcast(ry.view(rows // L, L, C), pe)
    torch.cuda.synchronize()
    assert torch.equal(y, ry) and torch.equal(mean, rm.view(-1)) and torch.equal(rstd, rr.view(-1))
    assert torch.equal(k, rk.view(rows, C))


def test_row_gate_cast_equals_cast_then_gate():
    """s2h_row_gate_cast (the low-res mask logits' fp32 cast + object-score gate, sam2_base.py:380-389):
    the bits of ops.cast + ops.row_gate forward, and of the gated gradient cast back to bf16"""
    from sam2_video.kernels import ops
    torch.manual_seed(8)
    x = torch.randn(13, 65536, device=DEV).to(torch.bfloat16)
    gate = torch.randn(13, device=DEV)
    gsave = torch.empty_like(gate)
    y = ops.row_gate_cast(x, gate, -1024.0, torch.float32, gate_out=gsave)
    ref = ops.row_gate(ops.cast(x, torch.float32), gate, -1024.0)
    g = torch.randn(13, 65536, device=DEV)
    dx = ops.row_gate_cast(g, gate, 0.0, torch.bfloat16, backward=True)
    rdx = ops.cast(ops.row_gate(g, gate, 0.0, backward=True), torch.bfloat16)
    torch.cuda.synchronize()
    assert torch.equal(y, ref) and torch.equal(gsave, gate) and torch.equal(dx, rdx)


def test_point_embed_grad_into_separate_rows():
    """s2h_point_embed_bwd_rows: the 5 label rows' gradients accumulated at their own addresses (the
    parameters' arena slices) -- the same additions in the same order as the table form"""
    from sam2_video.kernels import ops
    torch.manual_seed(9)
    R, D = 211, 256
    labels = torch.randint(-1, 4, (R,), device=DEV, dtype=torch.int32)
    dout = torch.randn(R, D, device=DEV).to(torch.bfloat16)
    base = torch.randn(5, D, device=DEV)
    rows = [torch.empty(D + 3, device=DEV)[k % 2:k % 2 + D] for k in range(5)]  # separate, ragged offsets
    for k in range(5):
        rows[k].copy_(base[k])
    table = base.clone()
    ops.point_embed_bwd_rows(labels, dout, rows)
    ops.point_embed_bwd(labels, dout, table)
    torch.cuda.synchronize()
    for k in range(5):
        assert torch.equal(rows[k], table[k])
