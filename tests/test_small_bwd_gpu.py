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
