"""The q / k projections' RoPE epilogues transposed into the flash backward's dQ / dK stores (round 5):
s2h_flash_bwd_frames_rope (memory self-attention queries, transformer.py:296-307 on the fused q/k/v
projection) and s2h_flash_bwd_frames_vfold_rope_qk (cross-attention queries and keys) against the
plain backward followed by the separate inverse rotation the fusion replaces (ops.rope_blocks,
frametape._linear_bw) -- within one bf16 rounding, rows past nrot and the untouched gradients
bit-identical -- and a bf16 training step with the fusion against S2H_BWD_ROPE_FUSE=0."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _close(a, b, tol, what=""):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    scale = b.abs().max().item() + 1e-6
    assert err <= tol * scale, f"{what}: max err {err:.3e} vs scale {scale:.3e} (tol {tol})"


def _tables(L):
    from sam2_video.model.modeling.position_encoding import axial_rope_table
    side = int(math.isqrt(L))
    return axial_rope_table(256, side, side, 10000.0, DEV)


@pytest.mark.parametrize("B,L,p_drop,keep", [(2, 1024, 0.1, True), (3, 256, 0.0, False), (2, 1024, 0.1, False)])
def test_flash_bwd_frames_rope_matches_separate_pass(B, L, p_drop, keep):
    from sam2_video.kernels import ops
    torch.manual_seed(7)
    F, H, D, seed = 3, 1, 256, 99
    bf = torch.bfloat16
    cos, sin = _tables(L)
    q = (torch.randn(F * B, L, H, D, device=DEV) * 0.5).to(bf)
    do = torch.randn(F * B, L, H, D, device=DEV).to(bf)
    k = (torch.randn(F * B * L, H, D, device=DEV) * 0.5).to(bf)
    v = torch.randn(F * B * L, H, D, device=DEV).to(bf)
    scale = D ** -0.5
    lks, krow, idx0 = [L] * F, [f * B * L for f in range(F)], [f * B * H * L * L for f in range(F)]
    nw = [ops.keep_words(B, H, L, L)] * F
    koff = [f * nw[0] for f in range(F)]
    kb = torch.zeros(F * nw[0], device=DEV, dtype=torch.int32)
    o, lse = torch.empty_like(q), torch.empty(F * B, H, L, device=DEV)
    for f in range(F):
        sl = slice(f * B, (f + 1) * B)
        kf, vf = k[krow[f]:krow[f] + B * L].view(B, L, H, D), v[krow[f]:krow[f] + B * L].view(B, L, H, D)
        ops.attn_fwd(q[sl], kf, vf, o[sl], lse[sl], scale, p_drop, seed, idx0=idx0[f],
                     keep=kb[koff[f]:koff[f] + nw[f]] if keep else None)
    kw = dict(keep=kb if keep else None, koff=koff if keep else None)
    out = {}
    for mode in ("plain", "q"):
        g = (torch.full_like(q, float("nan")), torch.full_like(k, float("nan")), torch.full_like(v, float("nan")))
        rope = (cos, sin, L, [L] * F) if mode == "q" else None
        ops.flash_bwd_frames(F, B, lks, krow, idx0, q, k, v, o, do, lse, *g, scale, p_drop, seed, rope=rope, **kw)
        torch.cuda.synchronize()
        out[mode] = g
    dq0, dk0, dv0 = out["plain"]
    ref_q = dq0.clone()
    ops.rope_blocks(ref_q.view(-1, D), (cos, sin, L, L, L, D, D), inverse=True)
    dq, dk, dv = out["q"]
    assert not torch.isnan(dq).any()
    assert torch.equal(dv, dv0) and torch.equal(dk, dk0)  # the key / value gradients are stored as before
    _close(dq, ref_q, 1e-2, "dq fused inverse rope vs separate pass")
    # bf16 ulp-level differences only (one rounding instead of two)
    assert (dq.float() - ref_q.float()).abs().max().item() <= 2 ** -6 * ref_q.float().abs().max().item()


@pytest.mark.parametrize("lks,nrots,p_drop", [([1028, 2060], [1024, 2048], 0.1), ([1024, 516], [1024, 512], 0.0)])
@pytest.mark.parametrize("variant", [1, 3])
def test_vfold_dq_store_applies_inverse_rope(lks, nrots, p_drop, variant):
    """the V-fold backward with the q projection's inverse RoPE in its dQ store (and the k projection's
    in the dK store) against the separate passes; variant 3 runs the one-wave 32x32 dK kernel, whose
    store carries the same rotation"""
    from sam2_video.kernels import ops
    from sam2_video.kernels._lib import lib
    B, Lq, seed = 2, 1024, 5
    bf = torch.bfloat16
    gen = torch.Generator(device="cpu").manual_seed(11)
    cos, sin = _tables(Lq)
    scale = 256 ** -0.5
    qs, ks, ms, us, lses, keeps, idx0, koff = [], [], [], [], [], [], [], []
    acc_e = acc_w = 0
    for lk in lks:
        q = (torch.randn(B, Lq, 1, 256, generator=gen) * 0.5).to(DEV, bf)
        k = (torch.randn(B, lk, 1, 256, generator=gen) * 0.5).to(DEV, bf)
        m = torch.randn(B, lk, 1, 64, generator=gen).to(DEV, bf)
        u = torch.empty(B, Lq, 1, 72, device=DEV, dtype=bf)
        lse = torch.empty(B, 1, Lq, device=DEV)
        keep = torch.zeros(ops.keep_words(B, 1, Lq, lk), device=DEV, dtype=torch.int32)
        ops.attn_fwd_vfold(q, k, m, u, lse, scale, p_drop, seed, idx0=acc_e, keep=keep if p_drop > 0 else None)
        idx0.append(acc_e)
        koff.append(acc_w)
        acc_e += B * Lq * lk
        acc_w += keep.numel()
        qs.append(q), ks.append(k.reshape(-1, 1, 256)), ms.append(m.reshape(-1, 1, 64)), us.append(u)
        lses.append(lse), keeps.append(keep)
    du = torch.randn(2 * B, Lq, 1, 72, generator=gen).to(DEV, bf)
    q_all, k_all, m_all = torch.cat(qs), torch.cat(ks), torch.cat(ms)
    krow = [0, B * lks[0]]
    kw = dict(keep=torch.cat(keeps) if p_drop > 0 else None, koff=koff if p_drop > 0 else None)
    out = {}
    prev = lib().s2h_attn_config(1)
    try:
        lib().s2h_attn_config(variant)
        for mode in ("plain", "k", "qk"):
            dq = torch.full_like(q_all, float("nan"))
            dk = torch.full_like(k_all, float("nan"))
            rope = None if mode == "plain" else (cos, sin, Lq, nrots)
            ops.flash_bwd_frames_vfold(2, B, lks, krow, idx0, q_all, k_all, m_all, torch.cat(us), du,
                                       torch.cat(lses), dq, dk, scale, p_drop, seed, rope=rope,
                                       rope_q=[Lq, Lq] if mode == "qk" else None, **kw)
            torch.cuda.synchronize()
            out[mode] = (dq, dk)
    finally:
        lib().s2h_attn_config(prev)
    dq0, dk0 = out["plain"]
    ref_q, ref_k = dq0.clone(), dk0.clone()
    ops.rope_blocks(ref_q.view(-1, 256), (cos, sin, Lq, Lq, Lq, 256, 256), inverse=True)
    for f, lk in enumerate(lks):
        ops.rope_blocks(ref_k[krow[f]:krow[f] + B * lk].view(-1, 256), (cos, sin, lk, nrots[f], Lq, 256, 256),
                        inverse=True)
    torch.cuda.synchronize()
    assert torch.equal(out["k"][0], dq0)  # dQ unrotated without rope_q
    assert torch.equal(out["k"][1], out["qk"][1])  # the dK store does not depend on rope_q
    _close(out["k"][1], ref_k, 1e-2, "dk fused vs separate")
    assert not torch.isnan(out["qk"][0]).any()
    _close(out["qk"][0], ref_q, 1e-2, "dq fused vs separate")
    for f, lk in enumerate(lks):  # the object-pointer key rows stay unrotated
        a_ = out["qk"][1][krow[f]:krow[f] + B * lk].view(B, lk, 256)[:, nrots[f]:]
        assert torch.equal(a_, dk0[krow[f]:krow[f] + B * lk].view(B, lk, 256)[:, nrots[f]:])


def test_step_rope_fusion_matches_separate_passes_bf16(monkeypatch):
    """a bf16 B+ 256^2 training step with the memory attention's inverse RoPE in the attention
    backward's stores (default) and as separate passes (S2H_BWD_ROPE_FUSE=0): the forward is the same
    (loss and logits bit-identical), gradients within bf16 rounding"""
    from step_harness import build_model, golden_batch, grads_by_name, load_golden, run_step
    g = load_golden("bplus256_point_all")
    batch = golden_batch(g).to(DEV)
    res = {}
    for flag in ("0", "1"):
        monkeypatch.setenv("S2H_BWD_ROPE_FUSE", flag)
        model = build_model("base_plus", 256, ["image_encoder", "memory_attention", "memory_encoder", "mask_decoder",
                                               "prompt_encoder"], "point", dtype="bf16")
        stages, merged, losses, _ = run_step(model, batch)
        res[flag] = ([s["pred_masks"].detach().float().cpu() for s in stages], float(losses["total_loss"]),
                     grads_by_name(model))
    (m0, l0, g0), (m1, l1, g1) = res["0"], res["1"]
    for a, b in zip(m0, m1):
        assert torch.equal(a, b)
    assert l0 == l1
    flat0 = torch.cat([v.flatten() for v in g0.values()]).double()
    flat1 = torch.cat([v.flatten() for v in g1.values()]).double()
    assert torch.nn.functional.cosine_similarity(flat0, flat1, dim=0).item() >= 0.999
    names = [n for n in g0 if "memory_attention" in n and (".q_proj." in n or ".k_proj." in n)]
    assert names
    worst = {}
    for n in names:
        cos = torch.nn.functional.cosine_similarity(g0[n].flatten().double(), g1[n].flatten().double(), dim=0).item()
        worst[n] = round(cos, 6)
    print("memory-attention q/k projection gradients, fused vs separate rope (cosine):", worst)
    for n, cos in worst.items():
        assert cos >= 0.99, (n, cos)
