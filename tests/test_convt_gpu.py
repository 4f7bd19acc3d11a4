"""ConvTranspose2d(2, 2) forward: the vectorised scatter with the bias and the residual add fused
(ops.convt2_store, mask_decoder.py:105-107 dc1(x) + feat_s1 / dc2(x) + feat_s0) against the scalar
scatter + separate add (bit-identical) and a torch fp32 reference."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("shape,add_batch", [((13, 32, 32, 256, 64), 1), ((13, 64, 64, 64, 32), 1),
                                              ((3, 5, 7, 32, 16), 3), ((2, 4, 4, 16, 8), 0)])
def test_convt2_store(dtype, shape, add_batch):
    from sam2_video.kernels import ops
    B, H, W, Ci, Co = shape
    torch.manual_seed(0)
    w32 = torch.randn(Ci, Co, 2, 2, device=DEV) / Ci ** 0.5
    w = w32.to(dtype).view(Ci, 4 * Co)
    bias = torch.randn(Co, device=DEV)
    x = torch.randn(B, H, W, Ci, device=DEV).to(dtype)
    add = torch.randn(add_batch, 2 * H, 2 * W, Co, device=DEV).to(dtype) if add_batch else None
    Y = torch.empty(B * H * W, 4 * Co, device=DEV, dtype=dtype)
    ops.gemm(x.reshape(-1, Ci), w, Y, M=B * H * W, N=4 * Co, K=Ci, lda_m=Ci, lda_k=1, ldb_k=4 * Co, ldb_n=1,
             ldc=4 * Co)
    out = ops.convt2_store(Y, B, H, W, Co, bias=bias, add=add)
    ref = ops.convt2_scatter(Y, B, H, W, Co, bias=bias)
    if add is not None:
        ref = ops.add(ref, add) if add_batch == B else ops.add_bcast(ref, add)
    torch.cuda.synchronize()
    t = torch.nn.functional.conv_transpose2d(x.float().permute(0, 3, 1, 2), w32.to(dtype).float(), bias,
                                             stride=2).permute(0, 2, 3, 1)
    if add is not None:
        t = t + add.float()
    # the same sums and roundings as the scatter + add launches
    assert torch.equal(out, ref)
    tol = 1e-2 if dtype == torch.bfloat16 else 1e-4
    assert (out.float() - t).abs().max().item() <= tol * t.abs().max().item()
