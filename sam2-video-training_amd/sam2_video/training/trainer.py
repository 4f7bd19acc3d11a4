"""SAM2LightningModule drop-in (reference sam2_video/training/trainer.py:28-322)
and the fit loop that replaces Lightning's (Lightning is not a dependency here).

Same constructor (model, loss, optimizer, scheduler, visualization config
sections), same loss selection, gt_stride, training_step/validation_step
signatures and logged keys.  `configure_optimizers` returns the arena AdamW
(eps/amsgrad of the YAML are ignored exactly as the reference does,
trainer.py:124-130) with the cosine-with-warmup schedule stepped per
optimizer step.  The reference's per-step torch.cuda.synchronize() +
empty_cache() (trainer.py:186-187) are host syncs with no effect on results and
are omitted.  W&B GIF logging is out of scope.
"""
from __future__ import annotations

import time
from types import SimpleNamespace
from typing import Any, Dict, List

import torch
from torch import nn

from ..eval.eval import evaluate_clip
from ..model.build import instantiate
from ..model.losses import CORE_LOSS_KEY, BCECategoryLoss, MultiStepMultiMasksAndIous
from .ddp import ArenaGradReducer
from .optim import ArenaAdamW, cosine_with_warmup


def _ns(x):
    if isinstance(x, dict):
        return SimpleNamespace(**{k: _ns(v) for k, v in x.items()})
    return x


def _get(ns, k, default=None):
    if isinstance(ns, dict):
        return ns.get(k, default)
    return getattr(ns, k, default)


def _todict(x):
    if isinstance(x, SimpleNamespace):
        return {k: _todict(v) for k, v in vars(x).items()}
    return x


class SAM2LightningModule(nn.Module):
    def __init__(self, model: Any, loss: Any, optimizer: Any, scheduler: Any, visualization: Any = None):
        super().__init__()
        self.hparams = SimpleNamespace(model=model, loss=_ns(loss), optimizer=_ns(optimizer),
                                       scheduler=_ns(scheduler), visualization=_ns(visualization or {}))
        self.model = None
        lt = _get(self.hparams.loss, "type", None)
        if lt is not None and str(lt).lower() in {"bce", "bce_only", "ce_only"}:
            self.criterion = BCECategoryLoss(pos_weight=_get(self.hparams.loss, "bce_pos_weight"),
                                             reduction=_get(self.hparams.loss, "bce_reduction", "mean"),
                                             logit_temperature=_get(self.hparams.loss, "bce_logit_temperature", 1.0))
        else:
            L = self.hparams.loss
            self.criterion = MultiStepMultiMasksAndIous(
                weight_dict=_todict(_get(L, "weight_dict")), supervise_all_iou=_get(L, "supervise_all_iou", False),
                iou_use_l1_loss=_get(L, "iou_use_l1_loss", False), pred_obj_scores=_get(L, "pred_obj_scores", False),
                focal_gamma_obj_score=_get(L, "focal_gamma_obj_score", 0.0),
                focal_alpha_obj_score=_get(L, "focal_alpha_obj_score", -1.0),
                logit_temperature=_get(L, "multistep_logit_temperature", 1.0))
        self.loss_gt_stride = max(int(_get(self.hparams.loss, "gt_stride", 1)), 1)
        self.logged: Dict[str, torch.Tensor] = {}
        self.optimizer = None
        self.lr_at = None
        self.reducer = None

    # ------------------------------------------------------------ setup
    def setup(self, stage: str = "fit", device=None):
        if stage == "fit":
            if self.model is None:
                m = self.hparams.model
                self.model = m if isinstance(m, nn.Module) else instantiate(_todict(m))
            self.model.load(device or "cuda")
            self.model.train()

    def configure_optimizers(self, total_steps: int = 1) -> Dict[str, Any]:
        o = self.hparams.optimizer
        if str(_get(o, "type", "adamw")).lower() == "adamw":
            opt = ArenaAdamW(self.model.arena, lr=_get(o, "lr", 1e-4), weight_decay=_get(o, "weight_decay", 0.01),
                             betas=tuple(_get(o, "betas", (0.9, 0.999))), eps=1e-8,
                             max_grad_norm=_get(o, "gradient_clip_val", 1.0))
        else:
            raise NotImplementedError("only AdamW (the reference configs' optimizer) is built")
        self.optimizer = opt
        sched = None
        if _get(self.hparams.scheduler, "enabled", True):
            total = max(1, int(total_steps))
            warm = total * float(_get(o, "warmup_factor", 0.0))
            if warm >= total:
                warm = max(0, total - 1)
            self.lr_at = cosine_with_warmup(opt.lr, warm, total, float(_get(self.hparams.scheduler, "num_cycles", 0.5)))
            sched = {"scheduler": self.lr_at, "interval": "step", "frequency": 1}
        return {"optimizer": opt, "lr_scheduler": sched} if sched else {"optimizer": opt}

    # --------------------------------------------------------- forward
    def forward(self, batch):
        return self.model(batch)

    def _apply_gt_stride(self, outs_per_frame, target_masks):
        """trainer.py:190-203"""
        if self.loss_gt_stride <= 1:
            return outs_per_frame, target_masks
        idxs = list(range(0, len(outs_per_frame), self.loss_gt_stride))
        return [outs_per_frame[i] for i in idxs], target_masks[idxs]

    def log(self, name, value, **kw):
        self.logged[name] = value.detach() if torch.is_tensor(value) else value

    def training_step(self, batch, batch_idx: int = 0) -> torch.Tensor:
        """trainer.py:256-289"""
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

    @torch.no_grad()
    def validation_step(self, batch, batch_idx: int = 0) -> torch.Tensor:
        """trainer.py:291-322 (loss, no gradient tape) plus the reference's offline evaluation
        metrics computed in the loop on every frame (eval/eval.py: IoU / Dice / MAE of the
        category-merged binarised masks, averaged as get_video_scores does): val/iou,
        val/dice, val/mae."""
        outs_per_frame, _ = self.forward(batch)
        outs, targets = self._apply_gt_stride(outs_per_frame, batch.masks)
        losses = self.criterion(outs, targets)
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
    """One optimizer step of the fit loop: zero grads -> training_step -> backward ->
    (RCCL all-reduce) -> clip + AdamW (+ schedule).  Everything stays on the device.

    graph=True captures zero-grad + forward + loss + backward of the step ONCE per input
    signature (frame count, image size, category/object layout) into a HIP graph and replays
    it: the ~6k kernel launches of a B+ 512^2 8-frame step cost one graph launch instead of
    ~6k Python/ctypes launches (the step was host-bound).  Per step, only the host prompt stage
    (connected components + clicks, sam2model.py:181-236), the copies of the new clip into the
    graph's static input buffers, the dropout RNG offset and the all-reduce + optimizer run
    eagerly.  Dropout masks still change every step: kernels fold the device-resident RNG
    offset into their seeds (s2h_rng_bind)."""

    def __init__(self, module: SAM2LightningModule, total_steps: int = 1, distributed: bool = False,
                 graph: bool = False):
        self.module = module
        module.configure_optimizers(total_steps)
        self.reducer = ArenaGradReducer(module.model.arena.grad_region()) if distributed else None
        self.global_step = 0
        self.graph = graph
        self._graphs: Dict[Any, Dict[str, Any]] = {}
        self.before_capture = None  # optional callable, run right before a graph is captured
        from ..kernels import functional as FN
        from ..kernels.ops import rng_offset
        self._fn = FN
        self.rng = rng_offset(module.model.arena.device)
        # every step (eager, warm-up, capture) draws the same per-launch host seeds; the step-to-step
        # variation of the dropout masks comes from the device RNG offset alone, so an eager step
        # and a replay of the captured one use identical masks
        self.seed_base = FN._SEED[0]

    def _device_step(self, batch):
        m = self.module
        self._fn.set_seed(self.seed_base)
        m.model.arena.zero_grad()
        loss = m.training_step(batch, self.global_step)
        loss.backward()
        return loss

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
            cur = torch.cuda.current_stream(dev)
            side = torch.cuda.Stream(dev)
            side.wait_stream(cur)
            with torch.cuda.stream(side):  # eager warm-up: fills every device-side table cache
                self._device_step(static)
            cur.wait_stream(side)
            if self.before_capture is not None:
                self.before_capture()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                loss = self._device_step(static)
            ent = self._graphs[key] = {"graph": g, "batch": static, "loss": loss, "logged": dict(self.module.logged),
                                       "outputs": self.module.last_outputs}
        else:
            st = ent["batch"]
            st.img_batch.copy_(batch.img_batch, non_blocking=True)
            st.masks.copy_(batch.masks, non_blocking=True)
            st.obj_to_frame_idx.copy_(batch.obj_to_frame_idx, non_blocking=True)
            model.upload_prompt_plan(plan, dev, out=st.prompt_plan["dev"])
            st.prompt_plan.update({k: plan[k] for k in ("points", "labels")})
        ent["graph"].replay()
        self.module.logged = dict(ent["logged"])
        self.module.last_outputs = ent["outputs"]
        return ent["loss"]

    def __call__(self, batch):
        m = self.module
        self.rng.fill_(self.global_step + 1)
        loss = self._graphed_step(batch) if self.graph else self._device_step(batch)
        scale = 1.0
        if self.reducer is not None:
            self.reducer.reduce()
            scale = self.reducer.grad_scale
        lr = m.lr_at(self.global_step) if m.lr_at is not None else None
        m.optimizer.step(lr=lr, grad_scale=scale)
        if m.optimizer is not None:
            m.log("train/learning_rate", m.optimizer.param_groups[0]["lr"])
        self.global_step += 1
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


def fit(module: SAM2LightningModule, batches, max_steps: int, device="cuda", log_every: int = 1, distributed=False,
        graph: bool = True):
    """Minimal fit loop (max_steps optimizer steps over an iterable of BatchedVideoDatapoint)."""
    module.setup("fit", device)
    run = StepRunner(module, max_steps, distributed, graph=graph)
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
