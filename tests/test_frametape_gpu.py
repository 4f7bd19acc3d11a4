"""Frame-batched backward of the tracking loop (kernels/frametape.py, model/tracking.py) against
the per-frame autograd path of the same build: the forward runs the same kernels in the same
order (dropout off), so outputs agree to the bit and gradients up to summation order; plus the
frame-table flash backward kernel against per-frame launches (dropout on, same masks)."""
import math

import numpy as np
import pytest
import torch

from step_harness import CASES, build_model, golden_batch, grads_by_name, load_golden, run_step

pytestmark = pytest.mark.gpu


def _pair(name, dtype):
    g = load_golden(name)
    size, prompt, trainable = CASES[name]
    out = []
    for batched in (False, True):
        m = build_model(size, int(g["meta/image_size"]), trainable, prompt, dtype=dtype, seed=int(g["meta/seed"]))
        m.frame_batched = batched
        batch = golden_batch(g).to("cuda")
        stages, merged, losses, _ = run_step(m, batch)
        out.append(([s["pred_masks"].detach().float().cpu() for s in stages],
                    {k: float(v) for k, v in losses.items() if torch.is_tensor(v)}, grads_by_name(m)))
        del m
    return out


@pytest.mark.parametrize("name", ["tiny256_point_all", "tiny256_point_mem", "bplus128_point_all_t8",
                                  "tiny256_mask_all", "tiny256_point_all_multi"])
def test_frame_batched_equals_per_frame_fp32(name):
    (la, lsa, ga), (lb, lsb, gb) = _pair(name, "fp32")
    for a, b in zip(la, lb):
        assert torch.equal(a, b)
    for k in lsa:
        assert abs(lsa[k] - lsb[k]) <= 1e-6 * max(1.0, abs(lsa[k])), (k, lsa[k], lsb[k])
    assert sorted(ga) == sorted(gb)
    # per parameter, relative to its own scale -- with a floor at 1e-6 of the largest gradient of
    # the step for the attention key biases, whose exact gradient is 0 (softmax shift invariance)
    gmax = max(float(g.abs().max()) for g in ga.values())
    bad = []
    for n in ga:
        ref = ga[n].double()
        err = (gb[n].double() - ref).abs().max().item()
        if err > 1e-5 * ref.abs().max().item() + 1e-6 * gmax:
            bad.append((n, err, ref.abs().max().item()))
    assert not bad, bad[:8]


def test_frame_batched_equals_per_frame_bf16(monkeypatch):
    """bf16 at B+ 256^2 (flash forward, frame-table flash backward, LDS-DMA GEMMs), dropout off:
    same forward bits; gradients within bf16 rounding of the per-frame path.  The decoder's fused
    token-side launches (tape only; their own check is tests/test_decoder_tok_gpu.py) and the mask
    head fused into the last upscaling launch (tape only, tests/test_convt_gpu.py) are off here: they
    compute the same ops in another fp32 summation order, so the forward bits would differ."""
    monkeypatch.setenv("S2H_DEC_TOK", "0")
    monkeypatch.setenv("S2H_CONVT_TAIL", "0")
    (la, lsa, ga), (lb, lsb, gb) = _pair("bplus256_point_all", "bf16")
    for a, b in zip(la, lb):
        assert torch.equal(a, b)
    assert abs(lsa["total_loss"] - lsb["total_loss"]) <= 1e-6 * abs(lsa["total_loss"])
    num = sum(float((gb[n].double() - ga[n].double()).norm() ** 2) for n in ga)
    den = sum(float(ga[n].double().norm() ** 2) for n in ga)
    rel = math.sqrt(num / den)
    print("global relative gradient difference batched vs per-frame (bf16):", rel)
    assert rel <= 2e-2, rel


@pytest.mark.parametrize("p_drop", [0.0, 0.1])
def test_flash_bwd_frames_matches_per_frame(p_drop):
    """s2h_flash_bwd_frames over 3 frames with packed K/V of 1028 / 2056 / 3084 keys vs one
    s2h_attn_bwd per frame with the same seed and index offsets"""
    from sam2_video.kernels import ops
    torch.manual_seed(0)
    B, Lq, H, D = 5, 256, 1, 256
    lks = [1028, 2056, 3084]
    F = len(lks)
    dt = torch.bfloat16
    q = (torch.randn(F * B, Lq, H, D, device="cuda") * 0.5).to(dt)
    do = torch.randn(F * B, Lq, H, D, device="cuda").to(dt)
    rows = sum(B * lk for lk in lks)
    k = (torch.randn(rows, H, D, device="cuda") * 0.5).to(dt)
    v = torch.randn(rows, H, D, device="cuda").to(dt)
    scale = 1.0 / math.sqrt(D)
    seed = 12345
    o = torch.empty_like(q)
    lse = torch.empty(F * B, H, Lq, device="cuda")
    krow, idx0, r, n = [], [], 0, 0
    for f, lk in enumerate(lks):
        krow.append(r)
        idx0.append(n)
        sl = slice(f * B, (f + 1) * B)
        ops.attn_fwd(q[sl], k[r:r + B * lk].view(B, lk, H, D), v[r:r + B * lk].view(B, lk, H, D), o[sl], lse[sl],
                     scale, p_drop, seed, idx0=n)
        r += B * lk
        n += B * H * Lq * lk
    dq_ref, dk_ref, dv_ref = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    for f, lk in enumerate(lks):
        sl = slice(f * B, (f + 1) * B)
        r0, r1 = krow[f], krow[f] + B * lk
        ops.attn_bwd(q[sl], k[r0:r1].view(B, lk, H, D), v[r0:r1].view(B, lk, H, D), o[sl], do[sl], lse[sl], dq_ref[sl],
                     dk_ref[r0:r1].view(B, lk, H, D), dv_ref[r0:r1].view(B, lk, H, D), scale, p_drop, seed,
                     idx0=idx0[f])
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    assert ops.flash_bwd_eligible(q)
    ops.flash_bwd_frames(F, B, lks, krow, idx0, q, k, v, o, do, lse, dq, dk, dv, scale, p_drop, seed)
    torch.cuda.synchronize()
    for a, b in ((dq, dq_ref), (dk, dk_ref), (dv, dv_ref)):
        err = (a.float() - b.float()).abs().max().item()
        assert err <= 2e-2 * b.float().abs().max().item(), err


def test_keep_bitmap_backward_equals_rehash():
    """the flash forward's dropout keep bitmap (s2h_attn_fwd keep) read by the backward gives the
    same gradients, bit for bit, as re-hashing every element: single launches (Lk not a multiple
    of 64) and the frame-table launch over packed per-frame bitmaps"""
    from sam2_video.kernels import ops
    torch.manual_seed(1)
    B, Lq, H, D, p, seed = 3, 256, 1, 256, 0.1, 777
    lks = [1028, 300, 2056]
    F = len(lks)
    dt = torch.bfloat16
    q = (torch.randn(F * B, Lq, H, D, device="cuda") * 0.5).to(dt)
    do = torch.randn(F * B, Lq, H, D, device="cuda").to(dt)
    rows = sum(B * lk for lk in lks)
    k = (torch.randn(rows, H, D, device="cuda") * 0.5).to(dt)
    v = torch.randn(rows, H, D, device="cuda").to(dt)
    scale = 1.0 / math.sqrt(D)
    assert ops.keep_bits_ok(q, p)
    nw = [ops.keep_words(B, H, Lq, lk) for lk in lks]
    koff = [sum(nw[:f]) for f in range(F)]
    keep = torch.full((sum(nw),), -1, device="cuda", dtype=torch.int32)
    o, o2 = torch.empty_like(q), torch.empty_like(q)
    lse, lse2 = torch.empty(F * B, H, Lq, device="cuda"), torch.empty(F * B, H, Lq, device="cuda")
    krow, idx0, r, n = [], [], 0, 0
    for f, lk in enumerate(lks):
        krow.append(r)
        idx0.append(n)
        sl = slice(f * B, (f + 1) * B)
        kf, vf = k[r:r + B * lk].view(B, lk, H, D), v[r:r + B * lk].view(B, lk, H, D)
        ops.attn_fwd(q[sl], kf, vf, o[sl], lse[sl], scale, p, seed, idx0=n, keep=keep[koff[f]:koff[f] + nw[f]])
        ops.attn_fwd(q[sl], kf, vf, o2[sl], lse2[sl], scale, p, seed, idx0=n)
        r += B * lk
        n += B * H * Lq * lk
    torch.cuda.synchronize()
    assert torch.equal(o, o2) and torch.equal(lse, lse2)
    # kept fraction over valid keys ~ 1 - p
    for f, lk in enumerate(lks):
        words = keep[koff[f]:koff[f] + nw[f]].view(B * H * Lq, -1).cpu().numpy().view("uint32")
        bits = ((words[:, :, None] >> np.arange(32, dtype=np.uint32)) & 1).reshape(B * H * Lq, -1)[:, :lk]
        assert abs(bits.mean() - (1 - p)) < 0.01, bits.mean()
    # single launches: bitmap vs re-hash
    for f, lk in enumerate(lks):
        sl = slice(f * B, (f + 1) * B)
        r0, r1 = krow[f], krow[f] + B * lk
        kf, vf = k[r0:r1].view(B, lk, H, D), v[r0:r1].view(B, lk, H, D)
        outs = []
        for kp in (keep[koff[f]:koff[f] + nw[f]], None):
            g = (torch.empty_like(q[sl]), torch.empty_like(kf), torch.empty_like(vf))
            ops.attn_bwd(q[sl], kf, vf, o[sl], do[sl], lse[sl], *g, scale, p, seed, idx0=idx0[f], keep=kp)
            outs.append(g)
        torch.cuda.synchronize()
        for a, b in zip(*outs):
            assert torch.equal(a, b), f"frame {f}: {(a.float() - b.float()).abs().max().item()}"
    # frame table: bitmap vs re-hash
    outs = []
    for kp in (keep, None):
        g = (torch.empty_like(q), torch.empty_like(k), torch.empty_like(v))
        ops.flash_bwd_frames(F, B, lks, krow, idx0, q, k, v, o, do, lse, *g, scale, p, seed, keep=kp,
                             koff=koff if kp is not None else None)
        outs.append(g)
    torch.cuda.synchronize()
    for a, b in zip(*outs):
        assert torch.equal(a, b), (a.float() - b.float()).abs().max().item()


@pytest.mark.parametrize("knob,fn", [("S2H_LN_BWD_FUSE", "linear_dgrad_ln_bwd"), ("S2H_LINEAR_LN", "linear_add_ln"),
                                     ("S2H_MLP_HEADS", "mlp_heads")])
def test_ln_fusions_equal_unfused(monkeypatch, knob, fn):
    """the fused per-object heads (S2H_MLP_HEADS, default on: the decoder's hypernetwork MLP and IoU
    head as one tape op and launch, kernels/frametape.mlp_heads) and the opt-in LayerNorm fusions of
    the memory attention against the separate launches, bf16 B+
    256^2: S2H_LN_BWD_FUSE=1 -- the LayerNorm backward in the dgrad of its output's only reader
    (frametape._ln_dgrad_fused: norm1 -> q/k/v, norm2 -> cross-attention q, norm3 -> linear1; same
    forward bits, gradients within the one bf16 rounding of dL/dt it skips); S2H_LINEAR_LN=1 -- the
    projection + residual add + LayerNorm in one full-row launch (s2h_linear_add_ln; the LayerNorm
    statistics in another summation order: forward and gradients within bf16 rounding)"""
    from sam2_video.kernels import ops
    calls = []
    orig = getattr(ops, fn)

    def counted(*a, **k):
        calls.append(1)
        return orig(*a, **k)
    monkeypatch.setattr(ops, fn, counted)
    g = load_golden("bplus256_point_all")
    size, prompt, trainable = CASES["bplus256_point_all"]
    out = []
    for fuse in ("0", "1"):
        monkeypatch.setenv(knob, fuse)
        m = build_model(size, int(g["meta/image_size"]), trainable, prompt, dtype="bf16", seed=int(g["meta/seed"]))
        m.frame_batched = True
        stages, merged, losses, _ = run_step(m, golden_batch(g).to("cuda"))
        out.append(([s["pred_masks"].detach().float().cpu() for s in stages], grads_by_name(m)))
        del m
        if fuse == "0":
            assert not calls
    assert calls, f"{fn} never ran"
    (la, ga), (lb, gb) = out
    for a, b in zip(la, lb):
        if knob in ("S2H_LN_BWD_FUSE", "S2H_MLP_HEADS"):  # the per-object heads are bit-identical too
            assert torch.equal(a, b)
        else:
            assert float((a - b).abs().max()) <= 3e-2 * float(a.abs().max()) + 1e-3
    num = sum(float((gb[n].double() - ga[n].double()).norm() ** 2) for n in ga)
    den = sum(float(ga[n].double().norm() ** 2) for n in ga)
    rel = math.sqrt(num / den)
    print(f"{knob}=1: {len(calls)} {fn} launches, global relative gradient difference {rel:.3e}")
    # LN_BWD_FUSE changes only the backward (measured 3.3e-4); LINEAR_LN changes the forward's LayerNorm
    # statistics' summation order, and the bf16 step carries that through 8 frames (measured 3.4e-2,
    # the per-frame vs frame-batched bf16 backward above differs by up to 2e-2)
    # S2H_MLP_HEADS: the same backward ops; only the order of the gradient adds into the decoder's
    # token rows differs
    assert rel <= {"S2H_LN_BWD_FUSE": 2e-2, "S2H_LINEAR_LN": 6e-2, "S2H_MLP_HEADS": 1e-3}[knob], rel
    for n in ga:
        if knob == "S2H_LN_BWD_FUSE" and n.startswith("memory_attention.") and ".norm" in n:
            r = float((gb[n].double() - ga[n].double()).norm() / (ga[n].double().norm() + 1e-12))
            assert r <= 5e-2, (n, r)


def test_wgrad_side_stream_equals_one_stream(monkeypatch):
    """the frame tapes' Linear weight gradients on a second stream (ops.SideWork, opt-in
    S2H_WGRAD_STREAM=1) against one stream: the same kernels on the same operands, so gradients agree up to the
    split-K atomics' summation order and the forward to the bit -- a missing fork / join or a
    buffer released to the allocator while the side stream still reads it would show here"""
    from sam2_video.kernels import ops
    g = load_golden("bplus256_point_all")
    size, prompt, trainable = CASES["bplus256_point_all"]
    out = []
    try:
        for on in (False, True):
            monkeypatch.setitem(ops._SIDE, "on", on)
            m = build_model(size, int(g["meta/image_size"]), trainable, prompt, dtype="bf16", seed=int(g["meta/seed"]))
            m.frame_batched = True
            stages, merged, losses, _ = run_step(m, golden_batch(g).to("cuda"))
            torch.cuda.synchronize()
            # with the side stream the deterministic workspace is switched off (ops._det_workspace_mode)
            assert ops._WG_WS["on"] == (not on)
            out.append(([s["pred_masks"].detach().float().cpu() for s in stages], grads_by_name(m)))
            del m
    finally:
        ops._det_workspace_mode(True)  # the default for the tests that follow
    (la, ga), (lb, gb) = out
    for a, b in zip(la, lb):
        assert torch.equal(a, b)
    gmax = max(float(t.abs().max()) for t in ga.values())
    bad = [(n, float((gb[n] - ga[n]).abs().max())) for n in ga
           if float((gb[n].double() - ga[n].double()).abs().max()) > 1e-4 * float(ga[n].abs().max()) + 1e-6 * gmax]
    assert not bad, bad[:8]


def test_ma_shared_qkv_equals_per_object(monkeypatch):
    """memory attention layer 0 with its norm1 + q/k/v GEMM once per frame and the result broadcast to
    the objects (S2H_MA_SHARED_QKV, default on: MemoryAttention.forward / MemoryAttentionLayer.sublayers;
    the q/k/v gradient summed over the objects before ONE dgrad / wgrad) against the per-object form,
    bf16 B+ 256^2 frame-batched step: the same forward values (LayerNorm and GEMM rows are
    row-independent), gradients within the one bf16 rounding of the object-summed dL/dqkv"""
    from sam2_video.kernels import frametape
    calls = []
    orig = frametape.expand_batch

    def counted(*a, **k):
        calls.append(a[1].shape)
        return orig(*a, **k)
    monkeypatch.setattr(frametape, "expand_batch", counted)
    g = load_golden("bplus256_point_all")
    size, prompt, trainable = CASES["bplus256_point_all"]
    out, ncalls = [], []
    for on in ("0", "1"):
        monkeypatch.setenv("S2H_MA_SHARED_QKV", on)
        calls.clear()
        m = build_model(size, int(g["meta/image_size"]), trainable, prompt, dtype="bf16", seed=int(g["meta/seed"]))
        m.frame_batched = True
        stages, merged, losses, _ = run_step(m, golden_batch(g).to("cuda"))
        out.append(([s["pred_masks"].detach().float().cpu() for s in stages], grads_by_name(m)))
        ncalls.append(len(calls))
        del m
    # one more broadcast (of the packed q/k/v) per memory-conditioned frame
    assert ncalls[1] > ncalls[0], ncalls
    (la, ga), (lb, gb) = out
    for a, b in zip(la, lb):
        assert float((a - b).abs().max()) <= 1e-2 * float(a.abs().max()) + 1e-3
    num = sum(float((gb[n].double() - ga[n].double()).norm() ** 2) for n in ga)
    den = sum(float(ga[n].double().norm() ** 2) for n in ga)
    rel = math.sqrt(num / den)
    print(f"S2H_MA_SHARED_QKV=1: {ncalls} broadcasts, masks equal: {all(torch.equal(a, b) for a, b in zip(la, lb))}, "
          f"global relative gradient difference {rel:.3e}")
    assert rel <= 2e-2, rel
