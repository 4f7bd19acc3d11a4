"""The Lightning drop-in at the bench workload: SAM2LightningModule driven by
Lightning 2.x automatic optimization (tests/lightning_stub.py restates its hook order; Lightning is
not installed in this image) with best.yaml's trainer section (gradient_clip_val 1.0,
accumulate_grad_batches 16, reference configs/best.yaml:105-106), against this build's StepRunner
on the same clips from the same weights.

Under a Lightning trainer, training_step replays the StepRunner's captured forward + loss + backward
graph (SAM2LightningModule._pl_graphed_step) and the backward hook is a no-op, so:
* the gradient arena at each optimizer step is bit-identical to the StepRunner's, and so are the
  parameters after the step (the same fused clip + AdamW with the same gradient scale);
* with precision=16's GradScaler the backward is seeded with the scale and Lightning's unscale_
  brings the arena back to the StepRunner's (a power-of-two scale: equal up to subnormals);
* the micro-step costs the same: the second window's wall time within a few % of the StepRunner's.
"""
import time

import pytest
import torch

from lightning_stub import lightning_fit, make_trainer
from test_configs_gpu import _clips, _module

pytestmark = pytest.mark.gpu

ACC = 16


def _runner_windows(clips):
    from sam2_video.training.trainer import StepRunner
    m = _module("base_plus", 512, lr=1e-4, clip=1.0)
    run = StepRunner(m, total_steps=2, graph=True, accumulate_grad_batches=ACC, gradient_clip_val=1.0)
    arena, grads, params, times = m.model.arena, [], [], []
    torch.cuda.synchronize()
    t = time.perf_counter()
    for i, c in enumerate(clips):
        run(c)
        if (i + 1) % ACC == 0:
            grads.append(arena.grad_region().clone())  # the window's gradients (kept until the next window)
            params.append(arena.data[: arena.n_grad].clone())
            torch.cuda.synchronize()
            now = time.perf_counter()
            times.append(now - t)
            t = now
    assert run.global_step == 2
    return grads, params, times


def _lightning_windows(clips, scaler=None):
    m = _module("base_plus", 512, lr=1e-4, clip=None)  # the clip comes from the Trainer
    tr = make_trainer(ACC, len(clips), 1.0, precision="16-mixed" if scaler else "bf16-mixed", scaler=scaler)
    m._trainer = tr
    arena, grads, params, times = m.model.arena, [], [], []
    torch.cuda.synchronize()
    t = [time.perf_counter()]

    def on_step(i):
        grads.append(arena.grad_region().clone())
        params.append(arena.data[: arena.n_grad].clone())
        torch.cuda.synchronize()
        now = time.perf_counter()
        times.append(now - t[0])
        t[0] = now
    opt = lightning_fit(m, tr, clips, on_step=on_step)
    assert opt.impl.step_count == 2 and len(m._pl_run._graphs) == 1
    return grads, params, times


def test_lightning_graph_path_equals_step_runner():
    clips = _clips(range(300, 300 + 2 * ACC), 8, 512, 13, 13)
    g_run, p_run, t_run = _runner_windows(clips)
    g_pl, p_pl, t_pl = _lightning_windows(clips)
    for w in range(2):
        assert torch.isfinite(g_run[w]).all()
        assert torch.equal(g_run[w], g_pl[w]), (w, float((g_run[w] - g_pl[w]).abs().max()))
        assert torch.equal(p_run[w], p_pl[w]), (w, float((p_run[w] - p_pl[w]).abs().max()))
    # the second window (graphs captured in the first): 16 micro-steps + one optimizer step each
    ratio = t_pl[1] / t_run[1]
    print(f"window wall time: StepRunner {t_run[1] * 1e3:.1f} ms, Lightning path {t_pl[1] * 1e3:.1f} ms, "
          f"ratio {ratio:.4f}")
    assert ratio <= 1.03, (t_run, t_pl)


def test_lightning_graph_path_with_grad_scaler():
    """precision=16: the backward seeded with GradScaler's scale (65536 = 2^16), unscale_ by Lightning,
    no inf: the same step as the StepRunner's"""
    clips = _clips(range(300, 300 + ACC), 8, 512, 13, 13)
    g_run, p_run, _ = _runner_windows(clips + clips)
    scaler = torch.amp.GradScaler("cuda", init_scale=2.0 ** 16)
    g_pl, p_pl, _ = _lightning_windows(clips + clips, scaler=scaler)
    for w in range(2):
        torch.testing.assert_close(g_pl[w], g_run[w], rtol=1e-6, atol=1e-30)
        torch.testing.assert_close(p_pl[w], p_run[w], rtol=1e-6, atol=1e-9)
    assert float(scaler.get_scale()) == 2.0 ** 16  # no inf: no backoff (growth interval 2000)
