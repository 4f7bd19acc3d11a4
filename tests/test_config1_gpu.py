"""BASELINE config 1 end to end: the reference's own configs/overfit.yaml (Hiera-T,
use_activation_checkpoint :46, precision 16 :103, one train batch per epoch :112), composed into
tests/golden/overfit_cfg1.json by oracle/gen_config_golden.py (256^2, 2 synthetic 4-frame clips,
checkpoint_path null, 3 epochs), driven through `python -m sam2_video.train --config-json`
(train.main -> Trainer.fit -> StepRunner, captured graph).

BASELINE's `trainer.accelerator=cpu` is refused by this build: the reference cannot
run a GPU-less step either (its forward calls torch.cuda.synchronize(), trainer.py:186).

* fp32 mode (trainer.precision=32), dropout 0: the first optimizer step's logged total loss equals
  the reference's loss on the same clip and weights (tests/golden/tiny256_point_mem.pt, recorded by
  importing the reference: clip 7, Hiera-T 256^2, 4 frames, memory modules trainable), to the
  parity tolerance of tests/test_parity_gpu.py (1e-4 relative);
* the configured mode (precision 16 -> bf16, dropout 0.1 as trained): finite, within 8 % of the
  reference's dropout-free loss on the first step (measured 3.6 %: the dropout masks), and the
  one-clip overfit loop lowers the loss over 3 epochs;
* use_activation_checkpoint: true is announced as a no-recompute notice at construction.
"""
import json
import math
import os

import pytest
import torch

from step_harness import GOLD, load_golden

pytestmark = pytest.mark.gpu

CFG = os.path.join(GOLD, "overfit_cfg1.json")


def _fit(tmp_path, overrides, dropout=None):
    from sam2_video import train
    from sam2_video.model.modeling.sam2_base import ActivationCheckpointNotice

    seen = {}

    def before_fit(module, dm, trainer):
        seen["trainer"] = trainer
        if dropout is not None:
            from sam2_video.training.trainer import precision_dtype
            module.compute_dtype = precision_dtype(trainer.precision)
            module.setup("fit", "cuda")  # instantiate the model section now to set the dropout
            module.model.set_dropout(dropout)

    with pytest.warns(ActivationCheckpointNotice):
        tr = train.main(["--config-json", CFG, "--run-dir", str(tmp_path)] + overrides, before_fit=before_fit)
    assert os.path.isfile(tmp_path / "checkpoints" / "last.ckpt")
    return [row["train/total_loss"] for row in tr.history], tr


def test_config1_overfit_fp32_matches_reference_loss(tmp_path):
    g = load_golden("tiny256_point_mem")
    losses, tr = _fit(tmp_path, ["trainer.precision=32"], dropout=0.0)
    ref = float(g["loss/total_loss"])
    print("config 1 fp32 losses", losses, "reference", ref)
    assert tr.global_step == 3 and len(losses) == 3
    assert abs(losses[0] - ref) <= 1e-4 * max(1.0, abs(ref)), (losses[0], ref)
    assert losses[-1] < losses[0]


def test_config1_overfit_as_configured(tmp_path):
    with open(CFG) as f:
        cfg = json.load(f)
    assert cfg["trainer"]["precision"] == 16 and cfg["model"]["use_activation_checkpoint"] is True
    g = load_golden("tiny256_point_mem")
    losses, tr = _fit(tmp_path, [])
    ref = float(g["loss/total_loss"])
    print("config 1 bf16 (dropout 0.1) losses", losses, "reference fp32", ref)
    assert tr.global_step == 3 and all(math.isfinite(x) for x in losses)
    assert tr.runner.module.model.compute_dtype == torch.bfloat16
    # dropout 0.1 draws masks the fp32 reference run (dropout 0) does not have: measured 3.6 % below
    assert abs(losses[0] - ref) <= 0.08 * abs(ref), (losses[0], ref)
    assert losses[-1] < losses[0]
