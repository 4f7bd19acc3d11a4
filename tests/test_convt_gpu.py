"""ConvTranspose2d(2, 2) forward stored straight into the NHWC output by two batched GEMMs
(ops.convt2_gemm, mask_decoder.py:105-107) against the GEMM + scatter pass and a torch fp32 reference."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("shape", [(13, 64, 64, 256, 64), (13, 128, 128, 64, 32), (3, 5, 7, 32, 16)])
def test_convt2_direct_store(dtype, shape):
    from sam2_video.kernels import functional as FN
    from sam2_video.kernels import ops
    from sam2_video.model.modeling.layers import ConvTranspose2x2
    B, H, W, Ci, Co = shape
    torch.manual_seed(0)
    mod = ConvTranspose2x2(Ci, Co)
    w32 = torch.randn(Ci, Co, 2, 2, device=DEV) / Ci ** 0.5
    mod.weight._s2h_compute = w32.to(dtype)
    mod.bias = torch.nn.Parameter(torch.randn(Co, device=DEV))
    FN.new_step()
    x = torch.randn(B, H, W, Ci, device=DEV).to(dtype)
    out = torch.empty(B, 2 * H, 2 * W, Co, device=DEV, dtype=dtype)
    ops.convt2_gemm(x, *mod.store_weight(), out)
    Y = torch.empty(B * H * W, 4 * Co, device=DEV, dtype=dtype)
    ops.gemm(x.reshape(-1, Ci), mod.compute_weight(), Y, M=B * H * W, N=4 * Co, K=Ci, lda_m=Ci, lda_k=1,
             ldb_k=4 * Co, ldb_n=1, ldc=4 * Co)
    ref = ops.convt2_scatter(Y, B, H, W, Co, bias=mod.bias.detach())
    torch.cuda.synchronize()
    t = torch.nn.functional.conv_transpose2d(x.float().permute(0, 3, 1, 2), w32.to(dtype).float(), mod.bias.detach(),
                                             stride=2).permute(0, 2, 3, 1)
    tol = 1e-2 if dtype == torch.bfloat16 else 1e-4
    assert (out.float() - t).abs().max().item() <= tol * t.abs().max().item()
    if dtype == torch.float32:  # same K order per output element: the two forms agree to the last bit
        assert torch.equal(out, ref)
    else:  # the scatter pass rounds the GEMM output to bf16 before the bias, the direct store once after
        err_direct = (out.float() - t).abs().mean().item()
        err_scatter = (ref.float() - t).abs().mean().item()
        assert err_direct <= err_scatter * 1.01, (err_direct, err_scatter)
    # a new weight generation rebuilds the reordered weight
    mod.weight._s2h_compute = (2 * w32).to(dtype)
    FN.new_step()
    ops.convt2_gemm(x, *mod.store_weight(), out)
    torch.cuda.synchronize()
    assert (out.float() - (2 * t - mod.bias.detach())).abs().max().item() <= 2 * tol * t.abs().max().item()
