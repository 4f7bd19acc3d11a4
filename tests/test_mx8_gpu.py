"""MX-fp8 kernels (BASELINE config 5) against the CPU oracle (oracle/mx8_oracle.py):
s2h_mx8_quant bit-exact (codes and scale words, row-major and transposed sources),
s2h_gemm_mx8 against an fp64 product of the dequantised operands (tolerance 6e-5 * sum|a*b|:
the block-scaled MFMA sums its 128-deep products below fp32 precision -- measured up to
1.5e-5 * sum|a*b| at K = 112, against 2e-6 for an fp32 chain), every tiling, the fused
epilogue, and ops.linear_mx8 / linear_dgrad_mx8 against the bf16 kernels they replace."""
import numpy as np
import pytest
import torch

from oracle import mx8_oracle as mx

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ops():
    from sam2_video.kernels import ops as o
    return o


def _data(rows, cols, seed, dtype=torch.bfloat16):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(rows, cols, generator=g) * torch.exp2(torch.randint(-12, 12, (rows, 1), generator=g).float())
    if cols > 64:
        x[rows // 2, 32:64] = 0.0  # an all-zero block
    return x.to(dtype)


@pytest.mark.parametrize("rows,cols", [(64, 128), (100, 112), (37, 1000), (512, 2048), (3, 8)])
def test_quant_bitexact(ops, rows, cols):
    x = _data(rows, cols, rows + cols)
    got = ops.mx8_quant(x.cuda())
    torch.cuda.synchronize()
    q, e8 = mx.quantize(x.float().numpy())
    assert np.array_equal(got.q.cpu().numpy(), q)
    assert np.array_equal(got.s.cpu().numpy(), mx.scale_words(e8))


@pytest.mark.parametrize("n,k", [(256, 112), (96, 300)])
def test_quant_transposed_bitexact(ops, n, k):
    w = _data(n, k, 7 * n + k).cuda()  # a weight [N, K]; quantise W^T [K, N] along N
    got = ops.mx8_quant(w, transpose=True)
    torch.cuda.synchronize()
    q, e8 = mx.quantize(w.float().cpu().numpy().T)
    assert np.array_equal(got.q.cpu().numpy(), q)
    assert np.array_equal(got.s.cpu().numpy(), mx.scale_words(e8))


def _deq(t, rows):
    return mx.dequantize(t.q.cpu().numpy(), mx.words_to_e8(t.s.cpu().numpy(), rows))


@pytest.mark.parametrize("cfg", [0, 1, 2, 3])
@pytest.mark.parametrize("M,N,K", [(200, 96, 112), (1000, 256, 256), (300, 2048, 256), (4096, 256, 2048)])
def test_gemm_mx8_exact_products(ops, M, N, K, cfg):
    from sam2_video.kernels._lib import lib
    a = ops.mx8_quant(_data(M, K, 1).cuda())
    b = ops.mx8_quant(_data(N, K, 2).cuda())
    c = torch.empty(M, N, device="cuda", dtype=torch.float32)
    prev = lib().s2h_mx8_config(cfg)  # returns the previous setting, not a status
    try:
        ops.gemm_mx8(a, b, c)
    finally:
        lib().s2h_mx8_config(prev)
    torch.cuda.synchronize()
    A, B = _deq(a, M), _deq(b, N)
    ref = A @ B.T
    bound = 6e-5 * (np.abs(A) @ np.abs(B).T) + 1e-30
    err = np.abs(c.cpu().numpy().astype(np.float64) - ref)
    assert (err <= bound).all(), float((err / bound).max())


def test_linear_mx8_epilogue(ops):
    M, N, K = 777, 448, 224
    x = (torch.randn(M, K) * 0.5).to(torch.bfloat16).cuda()
    w = (torch.randn(N, K) * 0.05).to(torch.bfloat16).cuda()
    bias = torch.randn(N).cuda()
    res = torch.randn(M, N).to(torch.bfloat16).cuda()
    w8 = ops.mx8_quant(w)
    pre = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    y = ops.linear_mx8(x, w8, bias, act="gelu", pre=pre)
    y2 = ops.linear_mx8(x, w8, bias, residual=res)
    torch.cuda.synchronize()
    X = torch.from_numpy(_deq(ops.mx8_quant(x), M)[:, :K])
    W = torch.from_numpy(_deq(w8, N)[:, :K])
    z = X @ W.T + bias.double().cpu()
    tol = dict(atol=2e-2, rtol=1e-2)  # bf16 outputs
    torch.testing.assert_close(pre.double().cpu(), z, **tol)
    torch.testing.assert_close(y.double().cpu(), torch.nn.functional.gelu(z), **tol)
    torch.testing.assert_close(y2.double().cpu(), z + res.double().cpu(), **tol)


def test_dgrad_mx8_matches_product(ops):
    M, N, K = 1024, 256, 448
    dy = (torch.randn(M, N) * 0.1).to(torch.bfloat16).cuda()
    w = (torch.randn(N, K) * 0.05).to(torch.bfloat16).cuda()
    wt8 = ops.mx8_quant(w, transpose=True)
    dx = ops.linear_dgrad_mx8(dy, wt8)
    torch.cuda.synchronize()
    D = _deq(ops.mx8_quant(dy), M)[:, :N]
    WT = _deq(wt8, K)[:, :N]
    ref = torch.from_numpy(D @ WT.T)
    torch.testing.assert_close(dx.double().cpu(), ref, atol=2e-3, rtol=1e-2)


def test_linear_mx8_close_to_bf16(ops):
    """fp8 quantisation error of a projection-shaped GEMM against the bf16 kernel: relative
    Frobenius error ~ e4m3's 2^-4 ulp averaged over K (measured ~2.5 %), bound 5 %"""
    M, N, K = 13312 // 4, 256, 256
    x = torch.randn(M, K).to(torch.bfloat16).cuda()
    w = (torch.randn(N, K) / 16).to(torch.bfloat16).cuda()
    y8 = ops.linear_mx8(x, ops.mx8_quant(w))
    y16 = ops.linear(x, w)
    torch.cuda.synchronize()
    rel = ((y8.float() - y16.float()).norm() / y16.float().norm()).item()
    assert rel < 0.05, rel
