"""Lightning `strategy` for running SAM2LightningModule under a real lightning.pytorch.Trainer on
several GPUs (the reference's `trainer.strategy=ddp`, README.md:155).

Lightning's DDPStrategy wraps the module in torch DistributedDataParallel, whose autograd hooks
wait for `param.grad` to be accumulated.  This build's backward kernels write the fp32 gradient
arena (kernels/arena.py) directly -- the parameters' `.grad` are views of it, autograd never
accumulates into them -- and the module's optimizer (training/optim.py ArenaOptimizer) all-reduces
the arena over RCCL (training/ddp.py) once per accumulation window, in its step.  `arena_ddp_strategy()` keeps
everything else of DDPStrategy -- process group, per-rank device, DistributedSampler injection,
rank-zero checkpointing -- and skips the wrapper.  Select it in the Hydra config:

    trainer:
      strategy:
        _target_: sam2_video.training.strategy.arena_ddp_strategy

Lightning is not installed in this image, so this class is exercised only through the stub-trainer
tests of the automatic-optimization path (tests/test_training_host.py); the build's own Trainer
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
