"""Lightning `strategy` for running SAM2LightningModule under a real lightning.pytorch.Trainer on
several GPUs (the reference's `trainer.strategy=ddp`, README.md:155).

Lightning's DDPStrategy wraps the module in torch DistributedDataParallel, which all-reduces
`param.grad`.  This build never fills `param.grad`: the backward kernels write the fp32 gradient
arena (kernels/arena.py) and SAM2LightningModule's manual-optimization runner all-reduces that
arena over RCCL (training/ddp.py) at accumulation boundaries.  `arena_ddp_strategy()` keeps
everything else of DDPStrategy -- process group, per-rank device, DistributedSampler injection,
rank-zero checkpointing -- and skips the wrapper.  Select it in the Hydra config:

    trainer:
      strategy:
        _target_: sam2_video.training.strategy.arena_ddp_strategy

Lightning is not installed in this image, so this class is exercised only through the stub-trainer
tests of the manual-optimization path (tests/test_training_host.py); the build's own Trainer
(training/trainer.py) is the tested multi-GPU driver.
"""
from __future__ import annotations


def arena_ddp_strategy(**kwargs):
    """DDPStrategy(**kwargs) that leaves the LightningModule unwrapped"""
    from lightning.pytorch.strategies import DDPStrategy

    class ArenaDDPStrategy(DDPStrategy):
        def configure_ddp(self) -> None:
            # no DistributedDataParallel: the module's gradient arena is reduced by its runner
            return None

    return ArenaDDPStrategy(**kwargs)
