"""The captured (HIP graph) training step against the eager one.

StepRunner(graph=True) captures zero-grad + forward + loss + backward once per input
signature and replays it; the prompt stage, the input copies, the dropout RNG offset and
the optimizer run eagerly.  Replays must reproduce the eager step on every clip (new data
through the static input buffers), and dropout masks must still change from step to step.
"""
import pytest
import torch

from step_harness import ALL

pytestmark = pytest.mark.gpu

LOSS = {"type": "multi_step", "gt_stride": 1, "multistep_logit_temperature": 1.0,
        "weight_dict": {"loss_mask": 20, "loss_dice": 1, "loss_iou": 1, "loss_class": 0},
        "supervise_all_iou": True, "iou_use_l1_loss": True, "pred_obj_scores": False}


def _runner(graph, dropout, lr=1e-4, dtype="fp32", size="tiny", S=128):
    from sam2_video.kernels import functional as FN
    from sam2_video.model.sam2model import SAM2Model
    from sam2_video.training.trainer import SAM2LightningModule, StepRunner
    FN.set_seed(777)  # the runner's per-step host seed base
    model = SAM2Model(None, f"{size}@{S}", trainable_modules=ALL, compute_dtype=dtype)
    model.set_dropout(dropout)
    opt = {"type": "AdamW", "lr": lr, "weight_decay": 0.01, "betas": [0.9, 0.999], "warmup_factor": 0.0}
    module = SAM2LightningModule(model, LOSS, opt, {"enabled": False})
    module.setup("fit", "cuda")
    return module, StepRunner(module, total_steps=4, graph=graph)


def _clips(idxs, T=3, S=128, n_cat=4, n_obj=3):
    from sam2_video.data.synthetic import make_clip, sam2_collate_fn
    return [sam2_collate_fn([make_clip(i, T, S, n_cat, n_obj)]).to("cuda") for i in idxs]


@pytest.mark.parametrize("dropout", [0.0, 0.1])
def test_graphed_steps_match_eager(dropout):
    """3 optimizer steps on 3 clips: per-step losses and logged values agree"""
    clips = _clips([11, 12, 13])
    out = []
    for graph in (False, True):
        module, run = _runner(graph, dropout)
        losses = [float(run(c).detach()) for c in clips]
        torch.cuda.synchronize()
        out.append((losses, {k: float(v) for k, v in module.logged.items() if torch.is_tensor(v)}))
        assert len(run._graphs) == (1 if graph else 0)
    (le, loge), (lg, logg) = out
    for a, b in zip(le, lg):
        assert abs(a - b) <= 1e-5 * max(1.0, abs(a)), (le, lg)
    for k in loge:
        assert abs(loge[k] - logg[k]) <= 1e-5 * max(1.0, abs(loge[k])), k


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("dropout", [0.0, 0.1])
def test_graphed_gradients_match_eager(dropout, dtype):
    """lr = 0 (weights fixed): every replayed step's gradient arena equals the eager step's BIT FOR BIT
    (round 5: no float atomics left in the gradient path -- the split-K weight gradients, column sums,
    LayerNorm parameter gradients and loss statistics reduce in a fixed order; round 4 allowed 1e-5 for
    their summation order)"""
    clips = _clips([14, 15])
    grads = []
    for graph in (False, True):
        module, run = _runner(graph, dropout, lr=0.0, dtype=dtype)
        g = []
        for c in clips:
            run(c)
            g.append(module.model.arena.grad_region().detach().clone())
        grads.append(g)
    for ge, gg in zip(*grads):
        assert torch.equal(ge, gg), (ge - gg).abs().max().item()


def test_graph_replays_draw_fresh_dropout_masks():
    """lr = 0 keeps the weights fixed, so replays of one clip differ only through dropout"""
    clip = _clips([21])[0]
    module, run = _runner(True, 0.1, lr=0.0)
    l1, l2 = float(run(clip).detach()), float(run(clip).detach())
    assert l1 != l2
    module0, run0 = _runner(True, 0.0, lr=0.0)
    m1, m2 = float(run0(clip).detach()), float(run0(clip).detach())
    assert abs(m1 - m2) <= 1e-6 * max(1.0, abs(m1))


def test_graph_recaptures_on_new_object_layout():
    module, run = _runner(True, 0.0)
    a = _clips([31], n_obj=3)[0]
    b = _clips([32], n_obj=2)[0]
    run(a)
    run(b)
    run(a)
    assert len(run._graphs) == 2
