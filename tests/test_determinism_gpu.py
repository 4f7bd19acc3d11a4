"""Bit-for-bit repeatability of the hot path on the GPU (round 4).

The SLP vectorizer's packed-fp32 code for the RoPE GEMM epilogue produced wrong values on one
16-lane quarter of a wave, intermittently, on gfx950 (csrc/Makefile: the library is now built with
-fno-slp-vectorize); the symptom was eager and replayed config-5 steps drifting apart from the first
memory-attention frame on.  These tests pin repeatability:

* single kernels at the step's shapes (the RoPE projection, the plain projection, flash and V-fold
  attention, add + LayerNorm), repeated with their output buffers pre-filled with garbage and the
  allocator's free memory overwritten: every repeat equals the first bit for bit;
* the training-mode forward of a whole clip (B+ 256^2, 4 frames, dropout 0.1 -- the same host seeds
  and device RNG offset) twice, with the allocator's free memory overwritten in between: every
  frame's logits bit-identical (the loss statistics' float atomics do not feed the logits).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _garble():
    x = torch.empty(1 << 30, dtype=torch.uint8, device=DEV)
    x.random_()
    del x


def _repeat(fn, outs, reps=12):
    ref = None
    for r in range(reps):
        for o in outs:
            if o.dtype.is_floating_point:
                o.fill_(float("nan") if r % 2 else 1e30)
            else:
                o.random_()
        if r % 3 == 2:
            _garble()
        fn()
        torch.cuda.synchronize()
        cur = [o.detach().clone() for o in outs]
        if ref is None:
            ref = cur
            continue
        for a, b in zip(ref, cur):
            assert torch.equal(a, b), f"repeat {r}: {int((a != b).sum())} elements differ"


def test_kernels_repeat_bitwise():
    from sam2_video.kernels import ops
    torch.manual_seed(0)
    bf = torch.bfloat16
    ops.rng_offset(DEV).fill_(3)
    O, L, C = 13, 1024, 256
    x = torch.randn(O * L, C, device=DEV).to(bf)
    w3 = (torch.randn(3 * C, C, device=DEV) * 0.06).to(bf)
    b3 = torch.randn(3 * C, device=DEV) * 0.1
    cos, sin = torch.randn(L, C // 2, device=DEV), torch.randn(L, C // 2, device=DEV)
    y3 = torch.empty(O * L, 3 * C, device=DEV, dtype=bf)
    _repeat(lambda: ops.linear_rope(x, w3, b3, (cos, sin, L, L, L, 2 * C, C), out=y3), [y3], reps=30)
    _repeat(lambda: ops.linear(x, w3, b3, out=y3), [y3])
    qkv = torch.randn(O, L, 3, 1, C, device=DEV).to(bf)
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    o = torch.empty(O, L, 1, C, device=DEV, dtype=bf)
    lse = torch.empty(O, 1, L, device=DEV)
    keep = torch.empty(ops.keep_words(O, 1, L, L), device=DEV, dtype=torch.int32)
    _repeat(lambda: ops.attn_fwd(q, k, v, o, lse, C ** -0.5, 0.1, 11, keep=keep), [o, lse, keep])
    Lk = 2060
    kk = torch.randn(O, Lk, 1, C, device=DEV).to(bf)
    mem = torch.randn(O, Lk, 1, 64, device=DEV).to(bf)
    u = torch.empty(O, L, 1, 72, device=DEV, dtype=bf)
    lse2 = torch.empty(O, 1, L, device=DEV)
    kp = torch.empty(ops.keep_words(O, 1, L, Lk), device=DEV, dtype=torch.int32)
    _repeat(lambda: ops.attn_fwd_vfold(q, kk, mem, u, lse2, C ** -0.5, 0.1, 13, keep=kp), [u, lse2, kp])
    g, bt = torch.randn(C, device=DEV), torch.randn(C, device=DEV)
    yl, xs = torch.empty(O * L, C, device=DEV, dtype=bf), torch.empty(O * L, C, device=DEV, dtype=bf)
    _repeat(lambda: ops.layernorm_fwd(x, g, bt, 1e-5, y=yl, add=x, xsum=xs), [yl, xs])


@pytest.mark.parametrize("dtype", ["bf16", "fp8"])
def test_training_forward_repeats_bitwise(dtype):
    from step_harness import ALL, build_model
    from test_configs_gpu import _clips
    from sam2_video.kernels import functional as FN
    from sam2_video.kernels.ops import rng_offset
    m = build_model("base_plus", 256, ALL, dtype=dtype, dropout=0.1)
    clip = _clips([70], 4, 256, 13, 13)[0]
    rng = rng_offset(m.arena.device)
    runs = []
    for r in range(3):
        if r:
            _garble()
        FN.set_seed(777)
        rng.fill_(1)
        out, _ = m(clip)
        torch.cuda.synchronize()
        runs.append([fr["pred_masks"].detach().clone() for fr in out])
        del out
    for r in (1, 2):
        for t, (a, b) in enumerate(zip(runs[0], runs[r])):
            assert torch.equal(a, b), (r, t, (a - b).abs().max().item())


@pytest.mark.parametrize("dtype", ["bf16", "fp8"])
def test_training_step_gradients_repeat_bitwise(dtype):
    """two eager forward + loss + backward steps of the same clip, weights and dropout draws (B+ 256^2,
    4 frames, dropout 0.1), the allocator's free memory overwritten in between: the whole gradient
    arena is bit-identical (round 5: the weight gradients' split-K reduction, the bias / LayerNorm /
    positional-table column sums and the loss statistics add per-workgroup partials in a fixed order
    instead of float atomics)"""
    from step_harness import ALL, build_model, run_step
    from test_configs_gpu import _clips
    from sam2_video.kernels import functional as FN
    from sam2_video.kernels.ops import rng_offset
    m = build_model("base_plus", 256, ALL, dtype=dtype, dropout=0.1)
    clip = _clips([70], 4, 256, 13, 13)[0]
    rng = rng_offset(m.arena.device)
    names = [(n, p) for n, p in m.named_parameters() if getattr(p, "_s2h_grad", None) is not None]
    grads, losses = [], []
    for r in range(3):
        if r:
            _garble()
        FN.set_seed(777)
        rng.fill_(1)
        _, _, lo, _ = run_step(m, clip)
        losses.append(float(lo["total_loss"].detach()))
        grads.append(m.arena.grad_region().clone())
    assert losses[0] == losses[1] == losses[2], losses
    for r in (1, 2):
        if not torch.equal(grads[0], grads[r]):
            diff = []
            for n, p in names:
                off = p._s2h_grad.data_ptr() - m.arena.grad.data_ptr()
                o, k = off // 4, p.numel()
                if not torch.equal(grads[0][o:o + k], grads[r][o:o + k]):
                    diff.append(n)
            raise AssertionError(f"run {r}: {len(diff)} parameters' gradients differ, e.g. {diff[:8]}")
