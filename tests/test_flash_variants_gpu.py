"""Round-6 flash kernel variants (s2h_flash_variant2 A/B bits): the head-dim-256 self-attention dQ kernel
with 8 fragment reads ahead (bit 1), the head-dim <= 128 dQ kernel (bit 2) and forward (bit 4) on the
3-stage LDS ring with one barrier per tile, the 32x32 dK / dV kernel on that ring (bit 8), the
one-row-per-wave key-split combine (bit 16).  Each computes the same sums in the same order as the
default kernel, so the outputs are bit-identical (forward O / LSE / keep bitmap, backward dQ / dK / dV),
with and without dropout (hashed, and the keep bitmap at head dim 256), with key and query tails."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("B,H,Lq,Lk,D,p", [(2, 2, 300, 260, 56, 0.1), (3, 1, 256, 200, 128, 0.0),
                                           (2, 1, 1024, 1024, 256, 0.1), (2, 2, 128, 70, 64, 0.0),
                                           (104, 1, 160, 300, 256, 0.1),
                                           (13, 1, 1024, 1024, 256, 0.1)])
def test_flash_round6_variants_bit_identical(B, H, Lq, Lk, D, p):
    from sam2_video.kernels import ops
    from sam2_video.kernels._lib import lib
    g = torch.Generator(device="cpu").manual_seed(3)
    bf = torch.bfloat16
    q = (torch.randn(B, Lq, H, D, generator=g) * 0.6).to(DEV, bf)
    k = (torch.randn(B, Lk, H, D, generator=g) * 0.6).to(DEV, bf)
    v = torch.randn(B, Lk, H, D, generator=g).to(DEV, bf)
    do = torch.randn(B, Lq, H, D, generator=g).to(DEV, bf)
    scale = D ** -0.5
    out = {}
    prev = lib().s2h_flash_variant2(-1)
    try:
        for bits in (0, 31):
            lib().s2h_flash_variant2(bits)
            o = torch.empty(B, Lq, H, D, device=DEV, dtype=bf)
            lse = torch.empty(B, H, Lq, device=DEV)
            keep = (torch.zeros(ops.keep_words(B, H, Lq, Lk), device=DEV, dtype=torch.int32)
                    if ops.keep_bits_ok(q, p) else None)  # the bitmap path: head dim 256
            ops.attn_fwd(q, k, v, o, lse, scale, p, 5, keep=keep)
            dq, dk, dv = (torch.full_like(t, float("nan")) for t in (q, k, v))
            ops.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, scale, p, 5, keep=keep)
            torch.cuda.synchronize()
            out[bits] = [o, lse, dq, dk, dv] + ([keep] if keep is not None else [])
    finally:
        lib().s2h_flash_variant2(prev)
    assert not torch.isnan(out[0][2].float()).any()
    for a, b in zip(out[0], out[31]):
        assert torch.equal(a, b)
