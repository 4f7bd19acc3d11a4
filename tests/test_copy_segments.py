"""ops.copy_segments (s2h_copy2d_batch): the memory bank assembly and gradient packing copies in one
launch.  Host: the 2-D reduction of (src, dst) layouts.  GPU: bit-identical to Tensor.copy_ for the
step's layouts (bank rows into a packed [O, M, C] buffer, flat gradient slices), ragged pairs in 4-B
pieces, 2-B ragged pairs through the Tensor.copy_ path, more than 16 pairs split over launches."""
import pytest
import torch


def _ops():
    from sam2_video.kernels import ops
    return ops


def test_pair_rows_layouts():
    ops = _ops()
    mem = torch.empty(13, 5 * 1024 + 64, 64, dtype=torch.bfloat16)
    f = torch.empty(13, 1024, 64, dtype=torch.bfloat16)
    # a bank entry: 13 rows of 1024 x 64 bf16, destination pitch = the packed buffer's object stride
    assert ops._pair_rows(f, mem[:, 1024:2048]) == (13, 1024 * 64 * 2, 1024 * 64 * 2, mem.stride(0) * 2)
    # contiguous on both sides: one row
    flat = torch.empty(4096, dtype=torch.float32)
    assert ops._pair_rows(flat[:1000], flat[2000:3000]) == (1, 4000, 4000, 4000)
    # size-1 dims are ignored; mismatched shapes and non-uniform pitches are refused
    assert ops._pair_rows(f[:1], mem[:1, :1024]) == (1, 1024 * 64 * 2, 1024 * 64 * 2, 1024 * 64 * 2)
    assert ops._pair_rows(f, mem[:, :1000]) is None
    x = torch.empty(4, 6, 8)
    assert ops._pair_rows(x[:, ::2], torch.empty(4, 3, 8)) == (12, 32, 64, 32)  # uniform pitch: one 2-D copy
    assert ops._pair_rows(x[:, :3, :4], torch.empty(4, 3, 4)) is None


@pytest.mark.gpu
def test_copy_segments_match_copy():
    ops = _ops()
    g = torch.Generator(device="cuda").manual_seed(7)
    O, C = 13, 64
    lens = [1024, 1024, 1024, 1024, 1024, 1024, 64]
    feats = [torch.randn(O, n, C, device="cuda", generator=g).bfloat16() for n in lens]
    M = sum(lens)
    got = torch.full((O, M, C), float("nan"), device="cuda", dtype=torch.bfloat16)
    ref = got.clone()
    r, pairs = 0, []
    for f in feats:
        pairs.append((f, got[:, r:r + f.shape[1]]))
        ref[:, r:r + f.shape[1]].copy_(f)
        r += f.shape[1]
    ops.copy_segments(pairs)
    torch.cuda.synchronize()
    assert torch.equal(got.view(torch.int16), ref.view(torch.int16))


@pytest.mark.gpu
def test_copy_segments_ragged_and_many():
    ops = _ops()
    g = torch.Generator(device="cuda").manual_seed(3)
    dst = torch.zeros(40000, device="cuda", dtype=torch.float32)
    ref = dst.clone()
    pairs, off = [], 0
    for i in range(21):  # > 16 pairs: two launches; sizes not multiples of 4 floats -> 4-B pieces
        n = 96 * (i + 1) + (3 if i % 5 == 4 else 0)
        src = torch.randn(n, device="cuda", generator=g)
        pairs.append((src, dst[off:off + n]))
        ref[off:off + n].copy_(src)
        off += n + (4 - n % 4) % 4
    ops.copy_segments(pairs)
    torch.cuda.synchronize()
    assert torch.equal(dst, ref)


def test_pair_rows_broadcast_source():
    """the decoder's learned tokens broadcast over the objects: a 2-D copy with source pitch 0"""
    ops = _ops()
    head = torch.empty(6, 256, dtype=torch.bfloat16)
    out = torch.empty(13, 8, 256, dtype=torch.bfloat16)
    assert ops._pair_rows(head.unsqueeze(0).expand(13, -1, -1), out[:, :6]) == (13, 6 * 512, 0, 8 * 512)


@pytest.mark.gpu
def test_copy_segments_broadcast_and_token_rows():
    """decoder_tokens' two copies (learned tokens to every object, source pitch 0; the prompt rows)
    and select_tokens' strided token reads in one launch each, bit-identical to Tensor.copy_"""
    ops = _ops()
    g = torch.Generator(device="cuda").manual_seed(5)
    O, nh, Ns, C = 13, 6, 2, 256
    head = torch.randn(nh, C, device="cuda", generator=g).bfloat16()
    sparse = torch.randn(O, Ns, C, device="cuda", generator=g).bfloat16()
    out = torch.full((O, nh + Ns, C), float("nan"), device="cuda", dtype=torch.bfloat16)
    ops.copy_segments([(head.unsqueeze(0).expand(O, -1, -1), out[:, :nh]), (sparse, out[:, nh:])])
    ref = torch.cat([head.unsqueeze(0).expand(O, -1, -1), sparse], 1)
    toks = [torch.empty(O, C, device="cuda", dtype=torch.bfloat16) for _ in range(2)]
    ops.copy_segments([(out[:, 1], toks[0]), (out[:, 2], toks[1])])
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    assert torch.equal(toks[0], ref[:, 1]) and torch.equal(toks[1], ref[:, 2])


@pytest.mark.gpu
def test_copy_segments_odd_bf16_falls_back():
    """a bf16 pair of odd length (not a 4-B multiple) goes through Tensor.copy_, beside batched pairs"""
    ops = _ops()
    g = torch.Generator(device="cuda").manual_seed(9)
    a = torch.randn(13, device="cuda", generator=g).bfloat16()
    b = torch.randn(13, 1, device="cuda", generator=g)  # 52 B: 4-B pieces
    da = torch.zeros(13, device="cuda", dtype=torch.bfloat16)
    db = torch.zeros(13, 1, device="cuda")
    ops.copy_segments([(a, da), (b, db)])
    torch.cuda.synchronize()
    assert torch.equal(da, a) and torch.equal(db, b)
