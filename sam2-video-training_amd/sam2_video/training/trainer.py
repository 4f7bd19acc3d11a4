"""SAM2LightningModule / SAM2LightningDataModule drop-ins (reference
sam2_video/training/trainer.py:28-400) and a Lightning-API Trainer for them.

* `SAM2LightningModule(model, loss, optimizer, scheduler, visualization)`: same
  constructor sections, loss selection (multi_step | bce), gt_stride,
  training_step / validation_step signatures and logged keys.  It subclasses
  `lightning.pytorch.LightningModule` when Lightning is importable, else
  `nn.Module`.  `configure_optimizers` returns the arena AdamW (eps/amsgrad of
  the YAML are ignored exactly as the reference does, trainer.py:124-130) with
  the cosine-with-warmup schedule stepped per optimizer step.
* `SAM2LightningDataModule(data, train_shuffle)`: DataLoaders of B == 1 clips
  collated by `sam2_collate_fn` (trainer.py:325-400); COCO files when the data
  section's paths exist, synthetic clips of the data section's shape otherwise.
* `Trainer(**cfg.trainer)`: the `lightning.pytorch.Trainer` arguments the
  reference configs set (best.yaml:98-113) -- max_epochs / max_steps,
  accumulate_grad_batches, gradient_clip_val (0 / None = no clip, as Lightning),
  precision, val_check_interval, num_sanity_val_steps, limit_*_batches -- and
  `fit(module, datamodule)`.  `model/build.py` resolves the configs'
  `_target_: lightning.pytorch.trainer.trainer.Trainer` to it when Lightning is
  not installed (it is not in this image).
* `StepRunner`: one micro-step of the fit loop on the device (captured HIP
  graph per input signature), RCCL all-reduce + clip + AdamW at accumulation
  boundaries.

The reference's per-step torch.cuda.synchronize() + empty_cache()
(trainer.py:186-187) are host syncs with no effect on results and are omitted.
W&B GIF logging is out of scope.
"""
from __future__ import annotations

import math
import os
import time
from types import SimpleNamespace
from typing import Any, Dict, List, Optional

import torch
from torch import nn

from ..eval.eval import evaluate_clip
from ..model.build import instantiate
from ..model.losses import CORE_LOSS_KEY, BCECategoryLoss, MultiStepMultiMasksAndIous
from .ddp import ArenaGradReducer
from .optim import ArenaAdamW, ArenaOptimizer, cosine_with_warmup

try:  # the reference's base classes when Lightning is installed (it is not in this image)
    import lightning.pytorch as _pl
    _ModuleBase, _DataBase, HAVE_LIGHTNING = _pl.LightningModule, _pl.LightningDataModule, True
except Exception:  # pragma: no cover - depends on the environment
    _ModuleBase, _DataBase, HAVE_LIGHTNING = nn.Module, object, False


def _ns(x):
    if isinstance(x, dict):
        return SimpleNamespace(**{k: _ns(v) for k, v in x.items()})
    return x


def _get(ns, k, default=None):
    if ns is None:
        return default
    if isinstance(ns, dict):
        return ns.get(k, default)
    return getattr(ns, k, default)


def _todict(x):
    if isinstance(x, SimpleNamespace):
        return {k: _todict(v) for k, v in vars(x).items()}
    if hasattr(x, "items") and not isinstance(x, dict):  # OmegaConf DictConfig
        return {k: _todict(v) for k, v in x.items()}
    return x


def precision_dtype(precision) -> str:
    """Lightning `precision` -> compute dtype of the kernels.  "16"/"16-mixed" (fp16 AMP in the
    reference configs, best.yaml:103) and "bf16*" run bf16 (same width; fp16 is not a CDNA4
    training format here), "32*"/"64*" run the fp32 mode, "fp8" / "transformer-engine" the MX-fp8
    mode."""
    p = str(precision if precision is not None else "bf16").lower()
    if p.startswith("fp8") or p.startswith("mxfp8") or p == "transformer-engine":
        return "fp8"  # MX-fp8 projections / FFN (BASELINE config 5, kernels/fp8.py)
    return "fp32" if p.startswith("32") or p.startswith("64") else "bf16"


class SAM2LightningModule(_ModuleBase):
    def __init__(self, model: Any, loss: Any, optimizer: Any, scheduler: Any, visualization: Any = None, *,
                 gradient_clip_val: Optional[float] = None, accumulate_grad_batches: Optional[int] = None):
        """The reference's five sections (trainer.py:38-99).  Under a Lightning Trainer the module uses
        Lightning's automatic optimization exactly as the reference does: the Trainer's
        gradient_clip_val and accumulate_grad_batches (best.yaml:105-106) apply as configured
        (configure_optimizers returns a torch.optim.Optimizer over the gradient arena,
        configure_gradient_clipping routes the clip into its fused kernel).  The two keyword-only
        extras are the same settings for this build's StepRunner when it is driven without a
        Trainer; this build's Trainer sets them from its own arguments."""
        super().__init__()
        cfg = SimpleNamespace(model=model, loss=_ns(_todict(loss)), optimizer=_ns(_todict(optimizer)),
                              scheduler=_ns(_todict(scheduler)), visualization=_ns(_todict(visualization or {})))
        if HAVE_LIGHTNING:  # pragma: no cover
            self.save_hyperparameters(ignore=["model"] if isinstance(model, nn.Module) else None)
        else:
            self.hparams = cfg
        self.cfg = cfg
        self.model = None
        L = cfg.loss
        lt = _get(L, "type", None)
        if lt is not None and str(lt).lower() in {"bce", "bce_only", "ce_only"}:
            self.criterion = BCECategoryLoss(pos_weight=_get(L, "bce_pos_weight"),
                                             reduction=_get(L, "bce_reduction", "mean"),
                                             logit_temperature=_get(L, "bce_logit_temperature", 1.0))
        else:
            self.criterion = MultiStepMultiMasksAndIous(
                weight_dict=_todict(_get(L, "weight_dict")), supervise_all_iou=_get(L, "supervise_all_iou", False),
                iou_use_l1_loss=_get(L, "iou_use_l1_loss", False), pred_obj_scores=_get(L, "pred_obj_scores", False),
                focal_gamma_obj_score=_get(L, "focal_gamma_obj_score", 0.0),
                focal_alpha_obj_score=_get(L, "focal_alpha_obj_score", -1.0),
                logit_temperature=_get(L, "multistep_logit_temperature", 1.0))
        self.loss_gt_stride = max(int(_get(L, "gt_stride", 1)), 1)
        self.logged: Dict[str, Any] = {}
        self.optimizer = None
        self.lr_at = None
        # clip / accumulation of the StepRunner (this build's Trainer overwrites them with its own
        # arguments; under Lightning the Trainer's own settings apply)
        self.gradient_clip_val = gradient_clip_val
        self.accumulate_grad_batches = accumulate_grad_batches
        self.compute_dtype = None  # set by the Trainer from `precision` (Lightning: setup reads it)

    # ------------------------------------------------------------ setup
    def setup(self, stage: str = "fit", device=None):
        """trainer.py:101-115: instantiate the model section, load it on the device (the current
        CUDA device -- the rank's own under DDP -- when none is given), train mode"""
        if stage == "fit":
            tr = self._attached_trainer()
            if self.compute_dtype is None and tr is not None and getattr(tr, "precision", None) is not None:
                self.compute_dtype = precision_dtype(tr.precision)  # Lightning's "16-mixed" etc.
            if self.model is None:
                m = self.cfg.model
                if isinstance(m, nn.Module):
                    self.model = m
                else:
                    kw = {"compute_dtype": self.compute_dtype} if self.compute_dtype else {}
                    self.model = instantiate(_todict(m), **kw)
            if device is None:
                device = torch.device("cuda", torch.cuda.current_device())
            self.model.load(device)
            self.model.train()

    def configure_optimizers(self, total_steps: Optional[int] = None) -> Optional[Dict[str, Any]]:
        """trainer.py:117-177: AdamW(lr, weight_decay, betas) -- eps 1e-8 / amsgrad False whatever the
        YAML says -- with get_cosine_schedule_with_warmup(total * warmup_factor, total), stepped per
        optimizer step.  The clip is the Trainer's gradient_clip_val (Lightning's clip_grad_norm_).
        Called by Lightning (no argument, a trainer attached): ArenaOptimizer, a torch.optim.Optimizer
        over the gradient arena, with a LambdaLR of that schedule over the trainer's
        estimated_stepping_batches (optimizer steps: Lightning counts them with its own
        accumulate_grad_batches and max_steps).  Called by StepRunner (total_steps given): the arena
        AdamW and the schedule as a step -> lr function."""
        o = self.cfg.optimizer
        if str(_get(o, "type", "adamw")).lower() != "adamw":
            raise NotImplementedError("only AdamW (the reference configs' optimizer) is built")
        tr = self._attached_trainer()
        if total_steps is None and tr is not None:
            return self._lightning_optimizers(tr)
        total_steps = 1 if total_steps is None else total_steps
        opt = ArenaAdamW(self.model.arena, lr=_get(o, "lr", 1e-4), weight_decay=_get(o, "weight_decay", 0.01),
                         betas=tuple(_get(o, "betas", (0.9, 0.999))), eps=1e-8,
                         max_grad_norm=self.gradient_clip_val)
        self.optimizer = opt
        sched = None
        if _get(self.cfg.scheduler, "enabled", True):
            total = max(1, int(total_steps))
            warm = total * float(_get(o, "warmup_factor", 0.0))
            if warm >= total:
                warm = max(0, total - 1)
            self.lr_at = cosine_with_warmup(opt.lr, warm, total, float(_get(self.cfg.scheduler, "num_cycles", 0.5)))
            sched = {"scheduler": self.lr_at, "interval": "step", "frequency": 1}
        return {"optimizer": opt, "lr_scheduler": sched} if sched else {"optimizer": opt}

    def _lightning_optimizers(self, tr) -> Dict[str, Any]:
        o = self.cfg.optimizer
        params = [p for p in self.model.parameters() if getattr(p, "_s2h_grad", None) is not None]
        lr = float(_get(o, "lr", 1e-4))
        acc = int(getattr(tr, "accumulate_grad_batches", 1) or 1)
        if self.accumulate_grad_batches not in (None, 1, acc):
            self._warn_once("acc", "SAM2LightningModule(accumulate_grad_batches=%s) is ignored under a Lightning "
                            "Trainer, whose accumulate_grad_batches=%s applies" % (self.accumulate_grad_batches, acc))
        opt = ArenaOptimizer(self.model.arena, params, lr=lr, weight_decay=_get(o, "weight_decay", 0.01),
                             betas=tuple(_get(o, "betas", (0.9, 0.999))), eps=1e-8,
                             max_grad_norm=getattr(tr, "gradient_clip_val", None) or 0.0)
        self.optimizer = opt
        if not _get(self.cfg.scheduler, "enabled", True):
            return {"optimizer": opt}
        total = max(1, int(getattr(tr, "estimated_stepping_batches", 1)))
        warm = total * float(_get(o, "warmup_factor", 0.0))
        if warm >= total:
            warm = max(0, total - 1)
        self.lr_at = cosine_with_warmup(lr, warm, total, float(_get(self.cfg.scheduler, "num_cycles", 0.5)))
        sched = torch.optim.lr_scheduler.LambdaLR(opt, lambda step: self.lr_at(step) / lr)
        return {"optimizer": opt, "lr_scheduler": {"scheduler": sched, "interval": "step", "frequency": 1}}

    def configure_gradient_clipping(self, optimizer, gradient_clip_val=None, gradient_clip_algorithm=None):
        """Lightning hook (automatic optimization, before each optimizer step): the Trainer's
        gradient_clip_val becomes the fused AdamW kernel's clip (clip_grad_norm_, norm type 2, on the
        device, no host sync) instead of torch's clip over every `p.grad`.  With no clip on the Trainer
        the module's own gradient_clip_val keyword (the StepRunner setting) applies, with a warning."""
        if gradient_clip_algorithm not in (None, "norm"):
            raise NotImplementedError("gradient_clip_algorithm='value' is not built (the reference clips by norm)")
        if gradient_clip_val is None and self.gradient_clip_val:
            self._warn_once("clip", "SAM2LightningModule(gradient_clip_val=%s) applies: the Lightning Trainer sets no "
                            "gradient_clip_val (set it on the Trainer, as best.yaml:105 does)" % self.gradient_clip_val)
            gradient_clip_val = self.gradient_clip_val
        opt = getattr(optimizer, "_optimizer", optimizer)  # LightningOptimizer wraps the optimizer
        opt.max_grad_norm = float(gradient_clip_val or 0.0)

    def _warn_once(self, key, msg):
        seen = self.__dict__.setdefault("_warned", set())
        if key not in seen:
            seen.add(key)
            import warnings
            warnings.warn(msg, UserWarning, stacklevel=3)

    def backward(self, loss, *args, **kwargs):
        """Lightning hook (automatic optimization): a no-op after the graph-replayed micro-step (its
        backward already filled the gradient arena inside training_step); otherwise loss.backward()
        with the gradient arena's deferred fixed-order sums flushed at its end
        (kernels.ops.deferred_grad_sums) and, on the last micro-batch of an accumulation window under
        DDP, the arena all-reduce -- before the precision plugin's GradScaler unscales and checks the
        gradients for inf / NaN, so every rank sees the same reduced gradients and takes the same
        skip-or-step decision (what DistributedDataParallel's in-backward reduce guarantees)"""
        if self.__dict__.pop("_pl_grads_ready", False):
            return
        from ..kernels.ops import deferred_grad_sums
        with deferred_grad_sums(self.model.arena.grad_region()):
            loss.backward(*args, **kwargs)
        if self.__dict__.pop("_pl_window_end", False):
            opt = self.optimizer
            if opt is not None and hasattr(opt, "reduce_now"):
                opt.reduce_now()

    # --------------------------------------------------------- forward
    def forward(self, batch):
        """trainer.py:182-188"""
        return self.model(batch)

    def _apply_gt_stride(self, outs_per_frame, target_masks):
        """trainer.py:190-203"""
        if self.loss_gt_stride <= 1:
            return outs_per_frame, target_masks
        idxs = list(range(0, len(outs_per_frame), self.loss_gt_stride))
        return [outs_per_frame[i] for i in idxs], target_masks[idxs]

    def log(self, name, value, **kw):
        self.logged[name] = value.detach() if torch.is_tensor(value) else value
        # not while a StepRunner records / captures the step: Lightning's metric updates would be
        # captured into the graph; the graph-replayed path logs the step's values after each replay
        if HAVE_LIGHTNING and self._attached_trainer() is not None and not self.__dict__.get("_in_runner"):
            super().log(name, value, batch_size=1, **kw)  # pragma: no cover

    # Under a Lightning Trainer (automatic optimization) training_step runs the whole micro-step --
    # forward, loss and the backward into the gradient arena -- as a replay of the captured HIP graph
    # (StepRunner's, the bench path) and returns the loss; the backward hook is then a no-op.  False:
    # the eager module (Lightning's own training_step -> backward order, no graph).
    lightning_graph = True

    def _pl_runner(self, tr, k):
        run = self.__dict__.get("_pl_run")
        if run is None or run.accumulate != k:
            import torch.distributed as dist
            world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
            run = StepRunner(self, graph=True, distributed=world > 1, accumulate_grad_batches=k, optimizer=False)
            self._pl_run = run
        return run

    @staticmethod
    def _pl_is_window_end(tr, batch_idx, k):
        """Lightning steps the optimizer after this micro-batch (fit_loop._should_accumulate() is
        False): the k-th batch of a window or the epoch's last batch"""
        loop = getattr(tr, "fit_loop", None)
        fn = getattr(loop, "_should_accumulate", None)
        if fn is not None:
            return not fn()
        n = getattr(tr, "num_training_batches", None)
        return (batch_idx + 1) % k == 0 or (isinstance(n, int) and batch_idx + 1 >= n)

    def _pl_graphed_step(self, batch, batch_idx, tr):
        """one Lightning micro-batch through the StepRunner: the arena is zeroed when the window starts
        (Lightning's zero_grad, which follows training_step in its closure, is then skipped for this
        micro-batch), the backward is seeded with the precision plugin's GradScaler scale (so
        unscale_ / the inf check see what loss.backward() of the scaled loss would have produced), and on
        the window's last micro-batch under DDP the arena ranges are all-reduced beside the staged
        backbone backward, as StepRunner overlaps them.  Lightning's 1/accumulate_grad_batches loss
        normalisation is folded into the optimizer step's gradient scale (ArenaOptimizer.window_scale),
        as StepRunner folds it: the arena holds the window's summed gradients, bit-identical to the
        StepRunner's."""
        k = max(1, int(getattr(tr, "accumulate_grad_batches", 1) or 1))
        run = self._pl_runner(tr, k)
        end = self._pl_is_window_end(tr, batch_idx, k)
        scaler = getattr(getattr(tr, "precision_plugin", None), "scaler", None)
        loss = run.lightning_micro_step(batch, window_start=batch_idx % k == 0, reduce=end, scaler=scaler)
        opt = self.optimizer
        if opt is not None:
            opt.hold_grads = batch_idx % k == 0  # the zero_grad Lightning issues after this training_step
            if end:
                opt.window_scale = 1.0 / k
                opt.reduced = run.reducer is not None
        self._pl_grads_ready = True
        if HAVE_LIGHTNING:  # pragma: no cover
            for name, v in self.logged.items():
                super().log(name, v, batch_size=1)
        return loss

    def training_step(self, batch, batch_idx: int = 0) -> torch.Tensor:
        """trainer.py:256-289: forward, the loss on the gt_stride frames, the logged terms; returns
        the loss (Lightning / StepRunner run the backward into the gradient arena).  Under a Lightning
        Trainer with lightning_graph (default) the micro-step is the StepRunner's graph replay
        (_pl_graphed_step)."""
        tr = self._attached_trainer()
        if tr is not None and not self.__dict__.get("_in_runner"):
            if self.lightning_graph:
                return self._pl_graphed_step(batch, batch_idx, tr)
            k = max(1, int(getattr(tr, "accumulate_grad_batches", 1) or 1))
            self._pl_window_end = self._pl_is_window_end(tr, batch_idx, k)
        outs_per_frame, obj_to_cat = self.forward(batch)
        self.last_outputs = outs_per_frame
        outs, targets = self._apply_gt_stride(outs_per_frame, batch.masks)
        losses = self.criterion(outs, targets)
        total = losses[CORE_LOSS_KEY]
        self.log("train/total_loss", total)
        for k, v in losses.items():
            if k in (CORE_LOSS_KEY, "logits"):
                continue
            self.log(f"train/{k}", v)
        if self.optimizer is not None:
            self.log("train/learning_rate", self.optimizer.param_groups[0]["lr"])
        return total

    def _attached_trainer(self):
        """the Lightning trainer driving this module (LightningModule._trainer), if any; this
        build's own Trainer drives StepRunner directly and does not attach itself"""
        return getattr(self, "_trainer", None)

    @torch.no_grad()
    def validation_step(self, batch, batch_idx: int = 0) -> torch.Tensor:
        """trainer.py:291-322 (loss, no gradient tape) in eval mode (dropout off, as Lightning's
        model.eval() before validation) plus the reference's offline evaluation metrics computed in
        the loop on every frame (eval/eval.py: IoU / Dice / MAE of the category-merged binarised
        masks, averaged as get_video_scores does): val/iou, val/dice, val/mae."""
        was = self.model.training
        self.model.eval()
        try:
            outs_per_frame, _ = self.forward(batch)
            outs, targets = self._apply_gt_stride(outs_per_frame, batch.masks)
            losses = self.criterion(outs, targets)
        finally:
            self.model.train(was)
        self.log("val/total_loss", losses[CORE_LOSS_KEY])
        for k, v in losses.items():
            if k not in (CORE_LOSS_KEY, "logits"):
                self.log(f"val/{k}", v)
        scores = evaluate_clip(outs_per_frame, batch.masks)
        self.last_eval = scores
        for k, v in scores["avg_scores"].items():
            self.log(f"val/{k}", v)
        return losses[CORE_LOSS_KEY]


class StepRunner:
    """One micro-step of the fit loop: (zero the arena when a window starts) -> training_step ->
    backward into the gradient arena, and at every `accumulate_grad_batches`-th micro-step: RCCL
    all-reduce (N > 1) -> clip + AdamW (+ schedule).  Everything stays on the device.

    Gradient accumulation follows Lightning: micro-step gradients are summed, the loss scale
    1/accumulate (and the 1/world average of DDP) is folded into the optimizer's grad_scale, the
    clip sees the scaled gradient, the schedule counts optimizer steps, and non-boundary
    micro-steps issue no all-reduce (DDP no_sync).

    graph=True captures forward + loss + backward of a micro-step ONCE per input signature
    (frame count, image size, category/object layout) into a HIP graph and replays it: the ~5k
    kernel launches of a B+ 512^2 8-frame step cost one graph launch instead of ~5k Python/ctypes
    launches.  Per step only the host prompt stage (connected components + clicks,
    sam2model.py:181-236), the copies of the new clip into the graph's static input buffers, the
    dropout RNG offset and the boundary work (all-reduce, optimizer, zeroing) run eagerly.
    Dropout masks still change every step: kernels fold the device-resident RNG offset into
    their seeds (s2h_rng_bind)."""

    def __init__(self, module: SAM2LightningModule, total_steps: int = 1, distributed: bool = False,
                 graph: bool = False, accumulate_grad_batches: int = 1, gradient_clip_val=None,
                 split_backward: Optional[bool] = None, optimizer: bool = True):
        """optimizer=False: the Lightning path (SAM2LightningModule._pl_graphed_step) -- the runner
        only runs micro-steps (lightning_micro_step); Lightning's optimizer loop steps the module's
        ArenaOptimizer"""
        self.module = module
        if gradient_clip_val is not None:
            module.gradient_clip_val = gradient_clip_val
        if optimizer:
            module.configure_optimizers(total_steps)
        arena = module.model.arena
        self.reducer = ArenaGradReducer(arena.grad_region(), split=arena.grad_split) if distributed else None
        # overlap: a two-phase backward -- (1) loss -> backbone outputs (the frame-batched
        # tracking backward completes every gradient except the backbone's), (2) the backbone's
        # backward in segments (SAM2Model.backbone_backward_segments: conv_s0/s1 + neck, then the
        # Hiera stages last to first) -- with the all-reduce of every completed arena range
        # (arena.grad_cuts) issued as soon as its segment ends, beside the following segments
        self.cuts = list(getattr(arena, "grad_cuts", [arena.grad_split, arena.n_grad]))
        split_ok = getattr(module.model, "frame_batched", False) and arena.grad_split < arena.n_grad
        self.overlap = bool(split_ok and (distributed if split_backward is None else split_backward))
        self.accumulate = max(1, int(accumulate_grad_batches or 1))
        self.global_step = 0  # optimizer steps
        self.micro_step = 0
        self.graph = graph
        self._graphs: Dict[Any, Dict[str, Any]] = {}
        self.before_capture = None  # optional callable, run right before a graph is captured
        from ..kernels import functional as FN
        from ..kernels.ops import deferred_grad_sums, rng_offset
        self._fn = FN
        self._sums = lambda: deferred_grad_sums(module.model.arena.grad_region())
        self.rng = rng_offset(module.model.arena.device)
        # every step (eager, warm-up, capture) draws the same per-launch host seeds; the step-to-step
        # variation of the dropout masks comes from the device RNG offset alone, so an eager step
        # and a replay of the captured one use identical masks
        self.seed_base = FN._SEED[0]
        self._pending = None
        self._segs = None
        # the backward's seed dL/dL: 1 (StepRunner), or the GradScaler scale of the Lightning path;
        # a device tensor read by the loss kernels' backward, so a captured graph picks up new values
        self.grad_seed = torch.ones((), device=arena.device, dtype=torch.float32)
        module.model.arena.zero_grad()

    def _device_step(self, batch):
        """forward + loss + backward (phase 1 only when overlapping; _phase2 finishes it)"""
        self._fn.set_seed(self.seed_base)
        m = self.module
        m._in_runner = True
        try:
            loss = m.training_step(batch, self.micro_step)
        finally:
            m._in_runner = False
        seed = self.grad_seed.view(loss.shape)
        bb = getattr(m.model, "last_backbone_outputs", None) if self.overlap else None
        with self._sums():  # each backward phase flushes its deferred gradient sums at its end
            if bb:
                grads = torch.autograd.grad(loss, bb, grad_outputs=seed, allow_unused=True)
                self._pending = [(t, g) for t, g in zip(bb, grads) if g is not None]
            else:
                self._pending = None
                loss.backward(seed)
        return loss

    def _segments(self):
        """the pending phase-2 backward as [(closure, arena rank)] (consumes the pending state)"""
        pend = self._pending
        self._pending = None
        if not pend:
            return []
        segs = getattr(self.module.model, "backbone_backward_segments", None)
        if segs is None:
            segs = [(lambda: torch.autograd.backward([t for t, _ in pend], [g for _, g in pend]), 0)]
        else:
            segs = segs(pend)

        def phase(run):
            def f():
                with self._sums():
                    run()
            return f
        return [(phase(run), rank) for run, rank in segs]

    def _phase2(self):
        for run, _ in self._segments():
            run()

    def _graphed_step(self, batch):
        model = self.module.model
        dev = model.arena.device
        plan = model.host_prompt_plan(batch)
        key = (tuple(batch.img_batch.shape), tuple(batch.masks.shape), tuple(plan["obj_to_cat"]),
               plan["num_categories"], tuple(t.shape for t in plan["host"]))
        ent = self._graphs.get(key)
        if ent is None:
            static = _static_batch(batch, dev)
            plan = dict(plan)
            plan["dev"] = model.upload_prompt_plan(plan, dev)
            static.prompt_plan = plan
            # the eager warm-up accumulates into the gradient arena: keep what earlier micro-steps
            # of this accumulation window left there
            saved = model.arena.grad_region().clone() if self.micro_step % self.accumulate else None
            cur = torch.cuda.current_stream(dev)
            side = torch.cuda.Stream(dev)
            side.wait_stream(cur)
            with torch.cuda.stream(side):  # eager warm-up: fills every device-side table cache
                self._device_step(static)
                self._phase2()
            cur.wait_stream(side)
            if saved is not None:
                model.arena.grad_region().copy_(saved)
            else:
                model.arena.zero_grad()
            if self.before_capture is not None:
                self.before_capture()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                loss = self._device_step(static)
            segs = []
            for run, rank in self._segments():  # the backbone's backward: one graph per segment
                gk = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gk, pool=g.pool()):
                    run()
                segs.append((gk.replay, rank, gk))
            ent = self._graphs[key] = {"graph": g, "segs": segs, "batch": static, "loss": loss,
                                       "logged": dict(self.module.logged), "outputs": self.module.last_outputs}
        else:
            st = ent["batch"]
            st.img_batch.copy_(batch.img_batch, non_blocking=True)
            st.masks.copy_(batch.masks, non_blocking=True)
            st.obj_to_frame_idx.copy_(batch.obj_to_frame_idx, non_blocking=True)
            model.upload_prompt_plan(plan, dev, out=st.prompt_plan["dev"])
            st.prompt_plan.update({k: plan[k] for k in ("points", "labels")})
        ent["graph"].replay()
        self._segs = [(rep, rank) for rep, rank, _ in ent["segs"]]
        self.module.logged = dict(ent["logged"])
        self.module.last_outputs = ent["outputs"]
        return ent["loss"]

    def begin_micro_step(self):
        """zero the gradient arena when an accumulation window starts (Lightning's zero_grad) and
        draw fresh dropout masks (the device RNG offset); shared by __call__ and the Lightning path"""
        if self.micro_step % self.accumulate == 0:
            self.module.model.arena.zero_grad()
        self.rng.fill_(self.micro_step + 1)
        self._fn.set_seed(self.seed_base)

    def flush(self) -> bool:
        """close a partial accumulation window (Lightning steps the optimizer on an epoch's last
        batch even when fewer than accumulate_grad_batches micro-steps were taken)"""
        if self.micro_step % self.accumulate == 0:
            return False
        self.micro_step += self.accumulate - self.micro_step % self.accumulate - 1
        return self.after_backward()

    def after_backward(self, reduced: bool = False) -> bool:
        """Counts the micro-step; at an accumulation boundary runs all-reduce (unless `reduced`:
        __call__ already overlapped it with the backward) + clip + AdamW (the arena is zeroed when
        the next window starts).  Returns True when an optimizer step was taken."""
        m = self.module
        self.micro_step += 1
        if self.micro_step % self.accumulate:
            return False
        scale = 1.0 / self.accumulate
        if self.reducer is not None:
            if not reduced:
                self.reducer.reduce()
            scale *= self.reducer.grad_scale
        lr = m.lr_at(self.global_step) if m.lr_at is not None else None
        m.optimizer.step(lr=lr, grad_scale=scale)
        m.log("train/learning_rate", m.optimizer.param_groups[0]["lr"])
        self.global_step += 1
        return True

    def __call__(self, batch):
        self.begin_micro_step()
        loss = self._run(batch, (self.micro_step + 1) % self.accumulate == 0)
        self.after_backward(reduced=self.overlap and self.reducer is not None
                            and (self.micro_step + 1) % self.accumulate == 0)
        return loss

    def lightning_micro_step(self, batch, window_start: bool, reduce: bool, scaler=None):
        """The Lightning path's micro-step (no optimizer step: Lightning's optimizer loop takes it):
        zero the arena when the accumulation window starts, draw fresh dropout masks, seed the backward
        with the GradScaler's current scale (device tensor, no host sync; its init_scale before the
        first scale() call; 1 without a scaler), forward + loss + backward (graph replay), and when
        `reduce` (the window's last micro-batch) under DDP the arena all-reduce of every range beside
        the staged backward, finished before this returns -- so Lightning's unscale_ / inf check /
        clip see the reduced gradients on every rank."""
        if window_start:
            self.module.model.arena.zero_grad()
        self.rng.fill_(self.micro_step + 1)
        self._fn.set_seed(self.seed_base)
        if scaler is not None and getattr(scaler, "is_enabled", lambda: True)():
            s = getattr(scaler, "_scale", None)
            if s is None:
                self.grad_seed.fill_(float(getattr(scaler, "_init_scale", 1.0)))
            else:
                self.grad_seed.copy_(s.reshape(()))
        else:
            self.grad_seed.fill_(1.0)
        loss = self._run(batch, reduce)
        if reduce and self.reducer is not None and not self.overlap:
            self.reducer.reduce()
        self.micro_step += 1
        return loss

    def _run(self, batch, boundary):
        """forward + loss + backward of one micro-step (graph replay or eager); at an accumulation
        boundary under DDP with the staged backward, each completed arena range is all-reduced beside
        the following segments (the works are waited for before this returns)"""
        self._segs = None
        loss = self._graphed_step(batch) if self.graph else self._device_step(batch)
        if self._segs is None:
            self._segs = self._segments()
        reduce = self.overlap and self.reducer is not None and boundary
        works = []
        if reduce:
            # the tracking gradients are complete: reduce them beside the backbone's backward
            works += self.reducer.reduce_range(0, self.cuts[0])
        done = 0  # arena ranks reduced so far
        for run, rank in self._segs:
            run()
            if reduce:  # this segment's range is complete: reduce it beside the next segments
                works += self.reducer.reduce_range(self.cuts[done], self.cuts[rank + 1])
                done = rank + 1
        self._segs = None
        if reduce:
            works += self.reducer.reduce_range(self.cuts[done], self.reducer.grad.numel())
            for w in works:
                w.wait()
        return loss


def _static_batch(batch, device):
    """device-resident copy of a batch whose tensors serve as a captured graph's input buffers"""
    from ..data.data_utils import BatchedVideoDatapoint
    out = BatchedVideoDatapoint(img_batch=batch.img_batch.to(device, copy=True),
                                obj_to_frame_idx=batch.obj_to_frame_idx.to(device, copy=True),
                                masks=batch.masks.to(device, copy=True), metadata=batch.metadata,
                                dict_key=batch.dict_key, batch_size=list(batch.batch_size))
    out.host_masks0 = None
    return out


# ------------------------------------------------------------------ data module
class SAM2LightningDataModule(_DataBase):
    """trainer.py:325-400: B == 1 clip DataLoaders collated by sam2_collate_fn.  The data section
    (configs/data/*.yaml: train_path, val_path, image_size, video_clip_length, stride,
    num_workers, batch_size, num_categories) is read as the reference reads it; when the COCO
    annotation files are not present the loaders yield deterministic synthetic clips of the same
    shape (data/synthetic.py): `synthetic_clips` per split, clip indices from
    `synthetic_{train,val}_offset` (default 0 / 100000), `synthetic_objects` objects."""

    def __init__(self, data: Any, train_shuffle: bool = True):
        if _DataBase is not object:  # pragma: no cover
            super().__init__()
        self.data = _ns(_todict(data))
        self.train_shuffle = train_shuffle
        self.hparams = SimpleNamespace(data=self.data, train_shuffle=train_shuffle)
        self.train_dataset = None
        self.val_dataset = None

    def _dataset(self, split):
        d = self.data
        path = _get(d, f"{split}_path")
        if path and os.path.exists(str(path)):
            from ..data.dataset import COCODataset
            return COCODataset(config=d, coco_json_path=path)
        from ..data.synthetic import SyntheticClipDataset
        n_cat = int(_get(d, "num_categories", 13))
        return SyntheticClipDataset(num_clips=int(_get(d, "synthetic_clips", 16 if split == "train" else 4)),
                                    num_frames=int(_get(d, "video_clip_length", 8)),
                                    image_size=int(_get(d, "image_size", 512)), n_cat=n_cat,
                                    n_obj=int(_get(d, "synthetic_objects", n_cat)),
                                    offset=int(_get(d, f"synthetic_{split}_offset", 0 if split == "train" else 100_000)))

    def setup(self, stage: str = "fit"):
        if stage == "fit":
            self.train_dataset = self._dataset("train")
            self.val_dataset = self._dataset("val")

    def _loader(self, ds, shuffle):
        """B == 1 clip loader; with more than one rank in the process group the clips are sharded
        by a DistributedSampler (what Lightning injects under strategy=ddp): every rank trains on
        its own clips, the Trainer calls sampler.set_epoch each epoch"""
        import torch.distributed as dist
        from torch.utils.data import DataLoader, DistributedSampler

        from ..data.synthetic import sam2_collate_fn
        if ds is None:
            raise RuntimeError("dataset not initialized: call setup('fit') first")
        sampler = None
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            sampler = DistributedSampler(ds, num_replicas=dist.get_world_size(), rank=dist.get_rank(),
                                         shuffle=shuffle)
        return DataLoader(ds, batch_size=int(_get(self.data, "batch_size", 1)),
                          num_workers=int(_get(self.data, "num_workers", 0)),
                          shuffle=shuffle if sampler is None else False, sampler=sampler,
                          pin_memory=torch.cuda.is_available(), collate_fn=sam2_collate_fn)

    def train_dataloader(self):
        return self._loader(self.train_dataset, self.train_shuffle)

    def val_dataloader(self):
        return self._loader(self.val_dataset, False)


# ---------------------------------------------------------------------- trainer
class Trainer:
    """The `lightning.pytorch.Trainer` surface the reference configs use (best.yaml:98-113), driving
    SAM2LightningModule through StepRunner.  Unknown Lightning arguments (logger, callbacks,
    enable_progress_bar, ...) are accepted and ignored."""

    def __init__(self, accelerator="auto", devices=1, precision=None, max_epochs=None, max_steps=-1,
                 gradient_clip_val=None, accumulate_grad_batches=1, val_check_interval=1.0,
                 num_sanity_val_steps=0, limit_train_batches=None, limit_val_batches=None,
                 log_every_n_steps=50, strategy="auto", graph=True, default_root_dir=None, **unused):
        if str(accelerator).lower() == "cpu":
            # the reference's config 1 (overfit.yaml, trainer.accelerator=cpu): this build's step is
            # HIP kernels only -- refuse rather than run on the GPU behind the caller's back
            raise ValueError("accelerator='cpu' is not supported: the sam2_video step runs as HIP kernels on an "
                             "MI355X (use accelerator='gpu' / 'auto')")
        self.accelerator = accelerator
        self.precision = precision
        self.devices = devices
        self.strategy = strategy
        self.max_epochs = max_epochs if max_epochs is not None else (1 if max_steps and max_steps > 0 else 1000)
        self.max_steps = int(max_steps if max_steps is not None else -1)
        self.gradient_clip_val = gradient_clip_val
        self.accumulate_grad_batches = max(1, int(accumulate_grad_batches or 1))
        self.val_check_interval = val_check_interval
        self.num_sanity_val_steps = int(num_sanity_val_steps or 0)
        self.limit_train_batches = limit_train_batches
        self.limit_val_batches = limit_val_batches
        self.log_every_n_steps = max(1, int(log_every_n_steps or 1))
        self.graph = graph
        self.default_root_dir = default_root_dir
        self.history: List[Dict[str, float]] = []
        self.val_history: List[Dict[str, float]] = []
        self.global_step = 0
        self.current_epoch = 0

    @staticmethod
    def _limit(n, lim):
        if lim is None:
            return n
        if isinstance(lim, float) and lim <= 1.0:
            return int(n * lim)
        return min(n, int(lim))

    def _validate(self, module, loader, device, n):
        vals = []
        for i, batch in enumerate(loader):
            if i >= n:
                break
            module.validation_step(batch.to(device, non_blocking=True), i)
            vals.append({k: float(v) for k, v in module.logged.items() if k.startswith("val/")})
        if vals:
            row = {k: sum(v[k] for v in vals) / len(vals) for k in vals[0]}
            row["step"] = self.global_step
            self.val_history.append(row)

    def fit(self, module: SAM2LightningModule, datamodule=None, train_dataloaders=None, val_dataloaders=None):
        from .ddp import init_from_env
        rank, world, local = init_from_env("nccl")
        device = torch.device("cuda", local)
        if world == 1:
            torch.cuda.set_device(device)
        if module.compute_dtype is None and self.precision is not None:
            module.compute_dtype = precision_dtype(self.precision)
        if datamodule is not None:
            datamodule.setup("fit")
            train_dataloaders = datamodule.train_dataloader()
            val_dataloaders = datamodule.val_dataloader()
        module.trainer_ = self
        module.setup("fit", device)
        n_train = self._limit(len(train_dataloaders), self.limit_train_batches)
        n_val = self._limit(len(val_dataloaders), self.limit_val_batches) if val_dataloaders is not None else 0
        # Lightning's estimated_stepping_batches: a partial last window is an optimizer step too
        per_epoch = max(1, math.ceil(n_train / self.accumulate_grad_batches))
        total = self.max_steps if self.max_steps > 0 else per_epoch * self.max_epochs
        run = StepRunner(module, total, distributed=world > 1, graph=self.graph,
                         accumulate_grad_batches=self.accumulate_grad_batches,
                         gradient_clip_val=self.gradient_clip_val)
        self.runner = run
        if n_val and self.num_sanity_val_steps:
            self._validate(module, val_dataloaders, device, min(n_val, self.num_sanity_val_steps))
            self.val_history.clear()
        vci = self.val_check_interval
        val_every = (max(1, int(n_train * vci)) if isinstance(vci, float) and vci <= 1.0 else int(vci)) if n_val else 0
        t0 = time.time()
        done = False
        for epoch in range(self.max_epochs):
            self.current_epoch = epoch
            sampler = getattr(train_dataloaders, "sampler", None)
            if hasattr(sampler, "set_epoch"):
                sampler.set_epoch(epoch)
            for i, batch in enumerate(train_dataloaders):
                if i >= n_train:
                    break
                before = run.global_step
                run(batch.to(device, non_blocking=True))
                self.global_step = run.global_step
                if run.global_step != before and run.global_step % self.log_every_n_steps == 0:
                    row = {k: float(v) for k, v in module.logged.items() if k.startswith("train/")}
                    row["step"], row["epoch"], row["time_s"] = run.global_step, epoch, time.time() - t0
                    self.history.append(row)
                if val_every and (i + 1) % val_every == 0:
                    self._validate(module, val_dataloaders, device, n_val)
                if self.max_steps > 0 and run.global_step >= self.max_steps:
                    done = True
                    break
            if done:
                break
            if run.flush():  # the epoch's last, partial accumulation window
                self.global_step = run.global_step
        return self.history

    def save_checkpoint(self, path, module: SAM2LightningModule):
        """Lightning-layout checkpoint: state_dict with the `model.` prefix (the reference strips it
        when it reloads, train.py:146-157) + optimizer state + counters.  Written by global rank 0
        only (Lightning's rank-zero checkpointing); the parameters are identical on every rank."""
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized() and dist.get_rank() != 0:
            return
        sd = {"model." + k: v.detach().cpu() for k, v in module.model.state_dict().items()}
        torch.save({"state_dict": sd, "optimizer_states": [module.optimizer.state_dict()],
                    "global_step": self.global_step, "epoch": self.current_epoch}, path)


def fit(module: SAM2LightningModule, batches, max_steps: int, device="cuda", log_every: int = 1, distributed=False,
        graph: bool = True, accumulate_grad_batches: int = 1, gradient_clip_val: Optional[float] = 1.0):
    """Minimal fit loop: `max_steps` micro-steps over an iterable of BatchedVideoDatapoint
    (gradient_clip_val 1.0 = best.yaml's trainer section)."""
    module.setup("fit", device)
    run = StepRunner(module, max(1, math.ceil(max_steps / max(1, accumulate_grad_batches))), distributed,
                     graph=graph, accumulate_grad_batches=accumulate_grad_batches,
                     gradient_clip_val=gradient_clip_val)
    hist: List[Dict[str, float]] = []
    t0 = time.time()
    for i, batch in enumerate(batches):
        if i >= max_steps:
            break
        run(batch.to(device, non_blocking=True))
        if (i + 1) % log_every == 0:
            row = {k: float(v) for k, v in module.logged.items()}
            row["step"] = i + 1
            row["time_s"] = time.time() - t0
            hist.append(row)
    return hist
