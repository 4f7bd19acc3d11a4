"""Lifetime rules of the captured step (a process abort reported during garbage
collection in test_config1_overfit_as_configured; DESIGN.md §10 round 6 has the analysis).

* A StepRunner's captured graphs -- the phase-1 graph and the backbone segment graphs that share its
  private memory pool (trainer.py `_graphed_step`) -- can be dropped and garbage-collected in any
  order while tensors from that pool (the static loss, the logged values) are still referenced; the
  pool's memory stays valid until the last of them goes, and a fresh runner on a fresh module then
  steps exactly as the first did.
* The buffers whose addresses libsam2hip keeps for the whole process (the RNG offset, the
  weight-gradient workspace, the deferral workspace) survive the teardown: the fresh runner's step
  reuses them.
Run at BASELINE config 1's shapes (Hiera-T, 256^2, 4 frames, bf16, dropout 0.1 as configured), the
configuration the abort was reported in.
"""
import gc
import math

import pytest
import torch

from test_configs_gpu import _clips, _module

pytestmark = pytest.mark.gpu


def _run(split, clips):
    from sam2_video.training.trainer import StepRunner
    m = _module("tiny", 256, dropout=0.1, lr=1e-4)
    run = StepRunner(m, total_steps=len(clips), graph=True, split_backward=split)
    losses = [run(c) for c in clips]
    return m, run, losses


@pytest.mark.parametrize("split", [False, True], ids=["one_graph", "segment_graphs_shared_pool"])
def test_runner_teardown_then_fresh_runner(split):
    from sam2_video.kernels import ops
    clips = _clips(range(7, 10), 4, 256, 3, 3)
    m, run, losses = _run(split, clips)
    assert (len(next(iter(run._graphs.values()))["segs"]) > 0) == split
    first = [float(x) for x in losses]
    keep = losses[-1]  # a tensor of the graphs' private pool, alive past the graphs
    logged = dict(m.logged)
    addrs = (ops.rng_offset("cuda").data_ptr(), ops._WG_WS["t"].data_ptr(), ops._DEFER["t"].data_ptr())
    del run, m, losses
    gc.collect()
    torch.cuda.synchronize()
    assert math.isfinite(float(keep)) and float(keep) == first[-1]
    assert all(torch.isfinite(v).all() for v in logged.values() if torch.is_tensor(v))
    del keep, logged
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    # fresh module + runner: the same weights, clips and RNG offsets give the same losses
    m2, run2, losses2 = _run(split, clips)
    second = [float(x) for x in losses2]
    torch.cuda.synchronize()
    assert addrs == (ops.rng_offset("cuda").data_ptr(), ops._WG_WS["t"].data_ptr(), ops._DEFER["t"].data_ptr())
    for a, b in zip(first, second):
        assert abs(a - b) <= 1e-6 * max(1.0, abs(a)), (first, second)
    del run2, m2, losses2
    gc.collect()
    torch.cuda.synchronize()


def test_graphs_released_before_their_outputs_and_in_reverse_capture_order():
    """the segment graphs released first, then the phase-1 graph whose pool they share, with the
    runner's outputs still referenced; then the outputs; every step in between synchronised"""
    clips = _clips(range(11, 13), 4, 256, 3, 3)
    m, run, losses = _run(True, clips)
    ent = next(iter(run._graphs.values()))
    outs = ent["outputs"]
    ref = float(losses[-1])
    run._segs = None
    for i in reversed(range(len(ent["segs"]))):
        ent["segs"].pop(i)
        gc.collect()
        torch.cuda.synchronize()
    del ent["graph"]
    gc.collect()
    torch.cuda.synchronize()
    assert float(losses[-1]) == ref
    run._graphs.clear()
    del run, ent
    gc.collect()
    torch.cuda.synchronize()
    assert outs is not None and float(losses[-1]) == ref
    del outs, losses, m
    gc.collect()
    torch.cuda.synchronize()
