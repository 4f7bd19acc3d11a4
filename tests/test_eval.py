"""Evaluation metrics (reference sam2_video/eval/eval.py): the CPU restatement (oracle/
eval_oracle.py) and this build's count-based scores against golden vectors produced by the
reference's own get_image_scores / get_video_scores / get_result (oracle/gen_eval_golden.py);
on the GPU, the HIP count kernel bit-exact against numpy and the in-loop clip evaluation of
the HIP model against the CPU oracle's (IoU within 1e-4, fp32 parity mode)."""
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
import eval_oracle as EO  # noqa: E402

GOLD = os.path.join(HERE, "golden", "eval_small.pt")
KEYS = ("iou", "mae", "dice")


def _golden():
    return torch.load(GOLD, weights_only=True)


def _table(s, n_cat):
    return np.array([[s["cat_scores"][c][k] for k in KEYS] for c in range(n_cat)], dtype=np.float64)


def _close(a, b, tol=1e-12):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    assert np.array_equal(np.isnan(a), np.isnan(b)), (a, b)
    m = ~np.isnan(a)
    assert np.allclose(a[m], b[m], rtol=tol, atol=tol), (a, b)


def _numpy_counts(pred_bin, gt):
    p, g = pred_bin.reshape(pred_bin.shape[0], -1), gt.reshape(gt.shape[0], -1)
    return np.stack([(p & g).sum(1), (p | g).sum(1), p.sum(1), g.sum(1)], 1).astype(np.int64)


def _split_frames(g):
    gt, dt = g["gt"].numpy(), g["dt"].numpy()
    return gt, dt, g["n_vid"], g["T"], gt.shape[1]


def test_oracle_matches_reference_eval():
    g = _golden()
    gt, dt, n_vid, T, n_cat = _split_frames(g)
    cats = list(range(n_cat))
    imgs = [EO.image_scores(dt[i], gt[i]) for i in range(n_vid * T)]
    for i, s in enumerate(imgs):
        _close(_table(s, n_cat), g["img_cat"][i].numpy())
        _close([s["avg_scores"][k] for k in KEYS], g["img_avg"][i].numpy())
    vids = [EO.video_scores(imgs[v * T:(v + 1) * T], cats) for v in range(n_vid)]
    for v, s in enumerate(vids):
        _close(_table(s, n_cat), g["video_cat"][v].numpy())
        _close([s["avg_scores"][k] for k in KEYS], g["video_avg"][v].numpy())
    r = EO.result(vids, cats)
    _close(_table(r, n_cat), g["result_cat"].numpy())
    _close([r["avg_scores"][k] for k in KEYS], g["result_avg"].numpy())


def test_count_based_scores_match_reference_eval():
    """the product's closed-form scores from the four integer counts (host aggregation)"""
    from sam2_video.eval import eval as E
    g = _golden()
    gt, dt, n_vid, T, n_cat = _split_frames(g)
    cats = list(range(n_cat))
    P = gt.shape[2] * gt.shape[3]
    imgs = [E.image_scores_from_counts(_numpy_counts(dt[i], gt[i]), P, cats) for i in range(n_vid * T)]
    for i, s in enumerate(imgs):
        _close(_table(s, n_cat), g["img_cat"][i].numpy(), 1e-9)
    vids = [E.get_video_scores_from_frames(imgs[v * T:(v + 1) * T], cats) for v in range(n_vid)]
    r = E.get_result(vids, cats)
    _close(_table(r, n_cat), g["result_cat"].numpy(), 1e-9)
    _close([r["avg_scores"][k] for k in KEYS], g["result_avg"].numpy(), 1e-9)


def test_reference_helpers_keep_their_semantics():
    from sam2_video.eval import eval as E
    g = _golden()
    gt, dt = g["gt"].numpy()[1], g["dt"].numpy()[1]
    m_dt, m_gt = E.merge_masks([dt[3]]), E.merge_masks([gt[3]])
    ref = g["img_cat"][1].numpy()[3]
    assert abs(E.caculate_iou(m_dt, m_gt) - ref[0]) < 1e-12
    assert abs(E.caculate_mae(m_dt, m_gt) - ref[1]) < 1e-12
    assert abs(E.caculate_dice(m_dt, m_gt) - ref[2]) < 1e-12


@pytest.mark.gpu
@pytest.mark.parametrize("N,H,W", [(13, 512, 512), (4, 37, 29), (1, 1, 1)])
def test_eval_counts_kernel_exact(N, H, W):
    from sam2_video.kernels import ops
    torch.manual_seed(N)
    logits = torch.randn(N, 1, H, W, device="cuda")
    logits[0] = -1.0  # an empty prediction
    gt = torch.rand(N, H, W, device="cuda") < 0.3
    got = ops.mask_eval_counts(logits, gt).cpu().numpy()
    ref = _numpy_counts((logits.cpu().numpy()[:, 0] > 0), gt.cpu().numpy())
    assert np.array_equal(got, ref)


@pytest.mark.gpu
def test_clip_evaluation_matches_oracle_fp32():
    """validation IoU of the HIP model (fp32 parity mode) vs the CPU oracle on the same clip"""
    import sam2_oracle as O
    from step_harness import ALL, build_model
    from sam2_video.data.synthetic import make_clip, sam2_collate_fn
    from sam2_video.eval.eval import evaluate_clip
    from sam2_video.model.configs import model_config
    from sam2_video.utils.init import synth_tensor

    size, S, T, n_cat, n_obj = "tiny", 128, 3, 4, 3
    clip = make_clip(5, T, S, n_cat, n_obj)
    model = build_model(size, S, ALL, "point", dtype="fp32")
    with torch.no_grad():
        merged, _ = model(sam2_collate_fn([clip]).to("cuda"))
    got = evaluate_clip(merged, clip["masks"].cuda())
    cfg = model_config(size, S)
    P = O.make_params(O.param_shapes(cfg), O.trainable_prefixes(ALL), synth_tensor, seed=0)
    _, o_merged, _ = O.OracleSAM2(cfg, P, dropout=0.0).forward(clip["images"], clip["masks"])
    cats = list(range(n_cat))
    imgs = [EO.image_scores((m["high_res"][:, 0] > 0).detach().numpy(), clip["masks"][t].numpy())
            for t, m in enumerate(o_merged)]
    ref = EO.video_scores(imgs, cats)
    for c in cats:
        for k in ("iou", "dice"):
            a, b = got["cat_scores"][c][k], ref["cat_scores"][c][k]
            assert (np.isnan(a) and np.isnan(b)) or abs(a - b) <= 1e-4, (c, k, a, b)
    assert abs(got["avg_scores"]["iou"] - ref["avg_scores"]["iou"]) <= 1e-4


@pytest.mark.gpu
def test_per_frame_backbone_for_eval_matches_batched():
    """forward_backbone_per_frame_for_eval (reference sam2model.py:164-169): in evaluation the image
    features of frame t are computed when the loop reaches frame t instead of for the whole clip up
    front -- the same per-frame masks (fp32 parity mode: the GEMM / attention results do not depend
    on how many frames share a launch)"""
    from step_harness import ALL, build_model
    from sam2_video.data.synthetic import make_clip, sam2_collate_fn

    clip = make_clip(7, 3, 128, 4, 3)
    model = build_model("tiny", 128, ALL, "point", dtype="fp32")
    model.eval()
    outs = []
    for flag in (False, True):
        model.forward_backbone_per_frame_for_eval = flag
        with torch.no_grad():
            merged, _ = model(sam2_collate_fn([clip]).to("cuda"))
        outs.append([m["pred_masks_high_res"].float().cpu() for m in merged])
    for a, b in zip(*outs):
        assert float((a - b).abs().max()) <= 1e-4 * max(1.0, float(a.abs().max())), float((a - b).abs().max())
