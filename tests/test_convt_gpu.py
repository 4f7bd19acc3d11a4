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


def test_convt2_tail_matches_three_launches():
    """dc2 + feat_s0, GELU and the hypernetwork mask product in one launch (s2h_convt2_tail,
    mask_decoder.py:105-113) against convt2_store + act_fwd + the batched GEMM: the saved pre / post
    activations bit-identical, the mask logits equal to the bf16 rounding of a differently ordered
    32-term fp32 sum"""
    from sam2_video.kernels import ops
    torch.manual_seed(3)
    B, H, W, Ci, Co = 13, 64, 64, 64, 32
    bf = torch.bfloat16
    w = (torch.randn(Ci, 4 * Co, device=DEV) / 8).to(bf)
    bias = torch.randn(Co, device=DEV) * 0.1
    x = torch.randn(B, H, W, Ci, device=DEV).to(bf)
    add = torch.randn(1, 2 * H, 2 * W, Co, device=DEV).to(bf)
    hyper = torch.randn(B, Co, device=DEV).to(bf)
    Y = torch.empty(B * H * W, 4 * Co, device=DEV, dtype=bf)
    ops.gemm(x.reshape(-1, Ci), w, Y, M=B * H * W, N=4 * Co, K=Ci, lda_m=Ci, lda_k=1, ldb_k=4 * Co, ldb_n=1,
             ldc=4 * Co)
    pre = torch.empty(B, 2 * H, 2 * W, Co, device=DEV, dtype=bf)
    post = torch.empty_like(pre)
    masks = torch.empty(B, 4 * H * W, device=DEV, dtype=bf)
    ops.convt2_tail(Y, B, H, W, Co, bias, add, hyper, pre, post, masks)
    ref_pre = ops.convt2_store(Y, B, H, W, Co, bias=bias, add=add)
    ref_post = ops.act_fwd(ref_pre, "gelu")
    ref_masks = torch.empty(B, 1, 4 * H * W, device=DEV, dtype=bf)
    ops.bmm(hyper.view(B, 1, Co), ref_post.view(B, -1, Co), ref_masks, trans_b=True)
    torch.cuda.synchronize()
    assert torch.equal(pre, ref_pre)
    assert torch.equal(post, ref_post)
    exact = (post.float().view(B, -1, Co) * hyper.float().view(B, 1, Co)).sum(-1)
    scale = exact.abs().max().item()
    assert (masks.float() - exact).abs().max().item() <= 8e-3 * scale
    assert (masks.float() - ref_masks.view(B, -1).float()).abs().max().item() <= 8e-3 * scale
    # at most a few bf16 ulps apart on a small fraction of the logits
    assert (masks != ref_masks.view(B, -1)).float().mean().item() < 0.05


def test_mask_decoder_tail_fused_matches_unfused_bf16(monkeypatch):
    """a bf16 B+ 256^2 training step with the mask decoder's dc2 / GELU / mask head fused (default) and
    as three launches (S2H_CONVT_TAIL=0): per-stage mask logits, loss and every gradient within bf16
    rounding of the mask logits' fp32 sum order"""
    from step_harness import build_model, golden_batch, grads_by_name, load_golden, mask_iou, run_step
    g = load_golden("bplus256_point_all")
    batch = golden_batch(g).to(DEV)
    res = {}
    for flag in ("0", "1"):
        monkeypatch.setenv("S2H_CONVT_TAIL", flag)
        model = build_model("base_plus", 256, ["image_encoder", "memory_attention", "memory_encoder", "mask_decoder",
                                               "prompt_encoder"], "point", dtype="bf16")
        stages, merged, losses, _ = run_step(model, batch)
        res[flag] = ([s["pred_masks"].detach().float().cpu() for s in stages], float(losses["total_loss"]),
                     grads_by_name(model))
    (m0, l0, g0), (m1, l1, g1) = res["0"], res["1"]
    for a, b in zip(m0, m1):
        assert mask_iou(a, b) >= 0.99
        assert (a - b).abs().max().item() <= 0.03 * b.abs().max().item()
    assert abs(l0 - l1) <= 3e-3 * abs(l0), (l0, l1)
    flat0 = torch.cat([v.flatten() for v in g0.values()]).double()
    flat1 = torch.cat([v.flatten() for v in g1.values()]).double()
    assert torch.nn.functional.cosine_similarity(flat0, flat1, dim=0).item() >= 0.999
    for n in ("sam_mask_decoder.output_upscaling.3.weight", "sam_mask_decoder.output_upscaling.3.bias",
              "sam_mask_decoder.output_hypernetworks_mlps.0.layers.2.weight"):
        cos = torch.nn.functional.cosine_similarity(g0[n].flatten().double(), g1[n].flatten().double(), dim=0).item()
        assert cos >= 0.99, (n, cos)


def test_convt2_ln_gelu_matches_three_launches():
    """dc1 + feat_s1, LayerNorm2d and GELU in one launch (s2h_convt2_ln_gelu, mask_decoder.py:105-106)
    against convt2_store + layernorm_fwd + act_fwd: every stored value bit-identical"""
    from sam2_video.kernels import ops
    from sam2_video.model.modeling.layers import LayerNorm2d
    torch.manual_seed(4)
    B, H, W, Ci, Co = 13, 32, 32, 256, 64
    bf = torch.bfloat16
    w = (torch.randn(Ci, 4 * Co, device=DEV) / 16).to(bf)
    bias = torch.randn(Co, device=DEV) * 0.1
    x = torch.randn(B, H, W, Ci, device=DEV).to(bf)
    add = torch.randn(1, 2 * H, 2 * W, Co, device=DEV).to(bf)
    ln = LayerNorm2d(Co).to(DEV)
    ln.weight.data = torch.randn(Co, device=DEV)
    ln.bias.data = torch.randn(Co, device=DEV)
    Y = torch.empty(B * H * W, 4 * Co, device=DEV, dtype=bf)
    ops.gemm(x.reshape(-1, Ci), w, Y, M=B * H * W, N=4 * Co, K=Ci, lda_m=Ci, lda_k=1, ldb_k=4 * Co, ldb_n=1,
             ldc=4 * Co)
    rows = B * 4 * H * W
    pre = torch.empty(B, 2 * H, 2 * W, Co, device=DEV, dtype=bf)
    y, post = torch.empty_like(pre), torch.empty_like(pre)
    mean, rstd = torch.empty(rows, device=DEV), torch.empty(rows, device=DEV)
    from sam2_video.kernels._lib import call
    call("s2h_convt2_ln_gelu", 1, B, H, W, Co, Y.data_ptr(), bias.data_ptr(), add.data_ptr(), 1,
         ln.weight.data_ptr(), ln.bias.data_ptr(), float(ln.eps), pre.data_ptr(), y.data_ptr(), mean.data_ptr(),
         rstd.data_ptr(), post.data_ptr(), ops.stream())
    ref_pre = ops.convt2_store(Y, B, H, W, Co, bias=bias, add=add)
    ref_y, ref_mean, ref_rstd = ops.layernorm_fwd(ref_pre, ln.weight.data, ln.bias.data, ln.eps)
    ref_post = ops.act_fwd(ref_y, "gelu")
    torch.cuda.synchronize()
    assert torch.equal(pre, ref_pre)
    assert torch.equal(mean, ref_mean.view(-1)) and torch.equal(rstd, ref_rstd.view(-1))
    assert torch.equal(y, ref_y)
    assert torch.equal(post, ref_post)


@pytest.mark.parametrize("dtype,Co", [(torch.bfloat16, 32), (torch.bfloat16, 64), (torch.float32, 16)])
def test_convt2_gather_vectorised(dtype, Co):
    """the backward's gather (vectorised, s2h_convt2 dir 1) is the exact inverse of the scatter and
    matches an index-built reference"""
    from sam2_video.kernels import ops
    torch.manual_seed(5)
    B, H, W = 13, 16, 24
    dout = torch.randn(B, 2 * H, 2 * W, Co, device=DEV).to(dtype)
    dY = ops.convt2_gather(dout, B, H, W, Co)
    ref = dout.view(B, H, 2, W, 2, Co).permute(0, 1, 3, 5, 2, 4).reshape(B * H * W, 4 * Co)
    torch.cuda.synchronize()
    assert torch.equal(dY, ref)
    assert torch.equal(ops.convt2_scatter(dY, B, H, W, Co), dout)
