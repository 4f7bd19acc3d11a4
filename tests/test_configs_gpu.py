"""The BASELINE.json configurations the bench and the scaling runs use, run on the GPU at their
full size (the oracle cannot finish them in seconds, so these check size-independent
properties):

* config 2 (B+, 512^2, 8 frames, 13 objects, bf16 -- the bench workload): finite losses, the
  captured HIP graph replayed 12 times (the regime where captured memset nodes once broke the
  stream order) reproduces the eager step clip by clip, and the bf16 mode stays
  close to the fp32 mode of the same build on the same clip;
* config 3 (B+, 384^2, 10 frames, 7 objects): the 10-frame bank and the graph path;
* config 4 (Hiera-L, 1024^2, 8 frames; 13 objects): head dim 72 on the padded-128 flash path,
  4096-token memory attention over a 7-frame bank (28k keys), the graph path;
* gradient accumulation (accumulate_grad_batches) equals the summed micro-step gradients;
* validation_step is deterministic (eval mode: dropout off).
"""
import math

import pytest
import torch

from step_harness import ALL, mask_iou

pytestmark = pytest.mark.gpu

LOSS = {"type": "multi_step", "gt_stride": 1, "multistep_logit_temperature": 1.0,
        "weight_dict": {"loss_mask": 20, "loss_dice": 1, "loss_iou": 1, "loss_class": 0},
        "supervise_all_iou": True, "iou_use_l1_loss": True, "pred_obj_scores": False}


def _module(size, S, dtype="bf16", dropout=None, lr=0.0, clip=1.0):
    from sam2_video.kernels import functional as FN
    from sam2_video.model.sam2model import SAM2Model
    from sam2_video.training.trainer import SAM2LightningModule
    FN.set_seed(4242)
    model = SAM2Model(None, f"{size}@{S}", trainable_modules=ALL, compute_dtype=dtype)
    if dropout is not None:
        model.set_dropout(dropout)
    opt = {"type": "AdamW", "lr": lr, "weight_decay": 0.01, "betas": [0.9, 0.999], "warmup_factor": 0.0}
    module = SAM2LightningModule(model, LOSS, opt, {"enabled": False})
    module.gradient_clip_val = clip
    module.setup("fit", "cuda")
    return module


def _clips(idxs, T, S, n_cat, n_obj):
    from sam2_video.data.synthetic import make_clip, sam2_collate_fn
    return [sam2_collate_fn([make_clip(i, T, S, n_cat, n_obj)]).to("cuda") for i in idxs]


def _losses(module, clips, graph):
    from sam2_video.training.trainer import StepRunner
    run = StepRunner(module, total_steps=len(clips), graph=graph)
    out = [float(run(c).detach()) for c in clips]
    torch.cuda.synchronize()
    return out, run


@pytest.mark.parametrize("cfg", [("base_plus", 512, 8, 13), ("base_plus", 384, 10, 7), ("large", 1024, 8, 13)],
                         ids=["config2", "config3", "config4"])
def test_config_graph_replays_match_eager(cfg):
    """lr = 0 (fixed weights), dropout 0.1 as trained: 12 replays (config 2) / 4 (config 3) / 2
    (config 4) of the captured step on different clips give the eager step's loss on each clip to
    1e-5 relative (the forward is bit-reproducible, tests/test_determinism_gpu.py)"""
    size, S, T, O = cfg
    n = {512: 12, 384: 4, 1024: 2}[S]
    clips = _clips(range(50, 50 + n), T, S, O, O)
    eager, _ = _losses(_module(size, S), clips, graph=False)
    graphed, run = _losses(_module(size, S), clips, graph=True)
    assert len(run._graphs) == 1
    assert all(math.isfinite(x) for x in eager + graphed), (eager, graphed)
    # fixed weights: the replay is the eager step bit for bit up to the loss statistics' float
    # atomics (summation order, ~1e-7); 1e-5 is the fp32-mode bound of test_graph_gpu.py
    for a, b in zip(eager, graphed):
        assert abs(a - b) <= 1e-5 * max(1.0, abs(a)), (eager, graphed)


def test_config2_bf16_close_to_fp32():
    """bf16 vs fp32 mode of this build on one config-2 clip (dropout off): binarised masks agree
    (IoU >= 0.97 per frame) and the loss within 2 % -- the size-independent counterpart of the
    golden bf16 test at 256^2"""
    from step_harness import run_step
    clip = _clips([77], 8, 512, 13, 13)[0]
    res = {}
    for dt in ("fp32", "bf16"):
        m = _module("base_plus", 512, dtype=dt, dropout=0.0)
        stages, merged, losses, _ = run_step(m.model, clip)
        res[dt] = ([s["pred_masks"].detach().float().cpu() for s in stages], float(losses["total_loss"]))
        del m, stages, merged
        torch.cuda.empty_cache()
    ious = [mask_iou(a, b) for a, b in zip(res["fp32"][0], res["bf16"][0])]
    errs = [(a - b).abs().max().item() for a, b in zip(res["fp32"][0], res["bf16"][0])]
    print("per-frame IoU bf16 vs fp32", ious, "max |dlogit|", errs, "losses", res["fp32"][1], res["bf16"][1])
    assert min(ious) >= 0.97, ious
    assert abs(res["fp32"][1] - res["bf16"][1]) <= 0.02 * abs(res["fp32"][1])


def _group_drift(a, b, names):
    """(relative RMS error |a - b| / |b|, cosine(a, b)) over the concatenated tensors `names`"""
    num = den = dot = na = 0.0
    for n in names:
        x, y = a[n].double(), b[n].double()
        num += float(((x - y) ** 2).sum())
        den += float((y ** 2).sum())
        dot += float((x * y).sum())
        na += float((x ** 2).sum())
    return math.sqrt(num / max(den, 1e-300)), dot / max(math.sqrt(na * den), 1e-300)


def test_config2_bf16_gradients_close_to_fp32():
    """the bench path's gradients at the bench size.  Config 2 (B+, 512^2, 8 frames,
    13 objects; dropout off), one clip: the bf16 gradient arena (V-fold cross-attention over banks of up
    to 7 x 1028 = 7196 keys, the fused decoder, every bench kernel) against this build's fp32 mode on
    the same clip and weights (the mode pinned to the reference at 128 / 256^2 by test_parity_gpu.py /
    test_training_step_gpu.py).  Per module group (step_harness.grad_group), over all its parameters:
    relative RMS error <= 2 x the reference's own bf16-vs-fp32 drift of that group at B+ 256^2 T = 8
    (tests/golden/bplus256_point_all_t8{,_bf16}.pt, its stored gradient tensors) + 0.02, and
    1 - cos <= 2 (1 - cos_ref) + 0.002; a mutated group (the memory attention's gradients x 1.15, a
    wrong dropout 1/keep scale) must fail the bound."""
    import collections

    from step_harness import grad_group, grads_by_name, load_golden, run_step
    clip = _clips([77], 8, 512, 13, 13)[0]
    grads = {}
    for dt in ("fp32", "bf16"):
        m = _module("base_plus", 512, dtype=dt, dropout=0.0)
        run_step(m.model, clip)
        grads[dt] = grads_by_name(m.model)
        del m
        torch.cuda.empty_cache()
    gf, gb = load_golden("bplus256_point_all_t8"), load_golden("bplus256_point_all_t8_bf16")
    ref_groups = collections.defaultdict(list)
    for k in gf:
        if k.startswith("grad/") and float(gf[k].double().norm()) > 0:
            ref_groups[grad_group(k[5:])].append(k[5:])
    gf = {k[5:]: v for k, v in gf.items() if k.startswith("grad/")}
    gb = {k[5:]: v for k, v in gb.items() if k.startswith("grad/")}
    ours_groups = collections.defaultdict(list)
    for n, g in grads["fp32"].items():
        if float(g.norm()) > 0:
            ours_groups[grad_group(n)].append(n)

    def check(bf16):
        bad, rows = [], []
        for grp, names in sorted(ours_groups.items()):
            e, c = _group_drift(bf16, grads["fp32"], names)
            if grp in ref_groups:
                e_ref, c_ref = _group_drift(gb, gf, ref_groups[grp])
            else:  # no stored reference tensor in this group: the worst group's drift
                e_ref, c_ref = max((_group_drift(gb, gf, v) for v in ref_groups.values()), key=lambda t: t[0])
            rows.append((grp, len(names), e, e_ref, 1 - c, 1 - c_ref))
            if e > 2 * e_ref + 0.02 or 1 - c > 2 * (1 - c_ref) + 0.002:
                bad.append(rows[-1])
        return rows, bad

    rows, bad = check(grads["bf16"])
    for r in rows:
        print("group %-40s n=%4d  rel-rms %.4f (ref %.4f)  1-cos %.2e (ref %.2e)" % r)
    assert not bad, bad
    # sensitivity: the memory attention's gradients off by 15 %
    mutated = dict(grads["bf16"])
    for n in ours_groups["memory_attention"]:
        mutated[n] = mutated[n] * 1.15
    _, bad_m = check(mutated)
    assert any(b[0] == "memory_attention" for b in bad_m), bad_m


def test_gradient_accumulation_sums_micro_steps():
    """accumulate_grad_batches = 2: the arena after two micro-steps equals the sum of the two
    single-step gradients (fp32, dropout off), no optimizer step in between"""
    from sam2_video.training.trainer import StepRunner
    clips = _clips([5, 6], 3, 128, 4, 3)
    single = []
    for c in clips:
        m = _module("tiny", 128, dtype="fp32", dropout=0.0)
        run = StepRunner(m, total_steps=1, graph=False, accumulate_grad_batches=1)
        m.optimizer.lr = 0.0
        run(c)
        single.append(m.model.arena.grad_region().detach().clone())
    for graph in (False, True):
        m = _module("tiny", 128, dtype="fp32", dropout=0.0)
        run = StepRunner(m, total_steps=1, graph=graph, accumulate_grad_batches=2)
        run(clips[0])
        assert run.global_step == 0
        run(clips[1])
        assert run.global_step == 1
        acc = m.model.arena.grad_region()
        ref = single[0] + single[1]
        assert (acc - ref).abs().max().item() <= 1e-5 * ref.abs().max().item(), graph


def test_validation_step_is_deterministic():
    """validation runs in eval mode (dropout off) and restores train mode"""
    m = _module("tiny", 128, dtype="bf16")
    clip = _clips([9], 3, 128, 4, 3)[0]
    vals = []
    for _ in range(2):
        m.validation_step(clip)
        vals.append({k: float(v) for k, v in m.logged.items() if k.startswith("val/")})
    assert m.model.training
    # equal up to the fp32 atomics of the loss reductions (summation order); dropout would
    # move them by far more
    for k in vals[0]:
        assert abs(vals[0][k] - vals[1][k]) <= 1e-5 * max(1.0, abs(vals[0][k])), (k, vals)


@pytest.mark.parametrize("graph", [False, True])
def test_split_backward_equals_single_backward(graph):
    """the staged backward of the DDP overlap (tracking gradients first, then the backbone's in
    segments -- conv_s0 / conv_s1 + neck, Hiera stages last to first -- one graph each) leaves the
    same gradient arena as one backward; the backbone's gradients sit at the arena tail
    (grad_split), conv_s0 / conv_s1 with them"""
    from sam2_video.training.trainer import StepRunner
    clips = _clips([3, 4], 3, 256, 4, 3)
    res = []
    for split in (False, True):
        m = _module("base_plus", 256, dtype="fp32", dropout=0.0)
        arena = m.model.arena
        names = [n for n in arena.grad_names if arena.offsets[n] >= arena.grad_split]
        assert names and all(n.startswith(("image_encoder.", "sam_mask_decoder.conv_s0.", "sam_mask_decoder.conv_s1."))
                             for n in names)
        assert any(n.startswith("sam_mask_decoder.conv_s0.") for n in names)
        run = StepRunner(m, total_steps=2, graph=graph, split_backward=split)
        assert run.overlap == split
        for c in clips:
            run(c)
        res.append(arena.grad_region().detach().clone())
    a, b = res
    assert (a - b).abs().max().item() <= 1e-5 * a.abs().max().item()


def test_lightning_checkpoint_resumes_on_device(tmp_path):
    """after a trained step, Trainer.save_checkpoint -> load_lightning_checkpoint into a fresh
    arena-backed model gives the trained weights (fp32 master copies and the bf16 shadow) and the
    same validation outputs on a clip (reference train.py:146-157 reloads checkpoints this way)"""
    from sam2_video.training.trainer import StepRunner, Trainer
    clip = _clips([21], 3, 128, 4, 3)[0]
    src = _module("tiny", 128, lr=1e-3)
    StepRunner(src, total_steps=1, graph=False)(clip)
    path = str(tmp_path / "last.ckpt")
    Trainer(max_steps=1).save_checkpoint(path, src)
    dst = _module("tiny", 128)
    dst.model.load_lightning_checkpoint(path)
    a, b = src.model.state_dict(), dst.model.state_dict()
    assert all(torch.equal(a[k], b[k]) for k in a)
    vals = []
    for m in (src, dst):
        m.validation_step(clip)
        vals.append({k: float(v) for k, v in m.logged.items() if k.startswith("val/")})
    for k in vals[0]:
        assert abs(vals[0][k] - vals[1][k]) <= 1e-5 * max(1.0, abs(vals[0][k])), (k, vals)
