"""Optimizer + schedule over the flat parameter arena.

ArenaAdamW = torch.optim.AdamW(trainable, lr, weight_decay, betas) as configured
by SAM2LightningModule.configure_optimizers (trainer.py:117-135: eps/amsgrad of
the YAML are NOT forwarded, so eps=1e-8, amsgrad=False) preceded by Lightning's
gradient_clip_val=1.0 (clip_grad_norm_, norm type 2).  One reduction kernel pair
computes the global norm and clip factor on the device; one fused kernel
applies clip + AdamW and refreshes the bf16 shadow weights -- no host sync.

Parameters whose gradient is None in the reference (never reached by the
step) are outside the gradient arena, so AdamW skips them exactly like torch.
"""
from __future__ import annotations

import math

import torch

from ..kernels import ops


class ArenaAdamW:
    def __init__(self, arena, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01, max_grad_norm=1.0):
        self.arena = arena
        self.lr = float(lr)
        self.betas = tuple(float(b) for b in betas)
        self.eps = float(eps)
        self.weight_decay = float(weight_decay)
        self.max_grad_norm = float(max_grad_norm) if max_grad_norm else 0.0
        self.step_count = 0
        dev = arena.device
        self._partial = torch.empty(1024, device=dev)
        self.norm_out = torch.zeros(2, device=dev)  # [grad norm, clip coefficient]
        self.param_groups = [{"lr": self.lr}]

    def step(self, lr=None, grad_scale=1.0):
        """grad_scale multiplies the stored gradients (1/world after a SUM all-reduce)"""
        a = self.arena
        if a.n_grad == 0:
            return
        self.step_count += 1
        if lr is not None:
            self.param_groups[0]["lr"] = float(lr)
        lr = self.param_groups[0]["lr"]
        g = a.grad_region()
        ops.grad_norm(g, self.max_grad_norm, self._partial, self.norm_out, grad_scale)
        shadow = a.shadow[: a.n_grad] if a.shadow is not None else None
        ops.adamw(a.data[: a.n_grad], g, a.exp_avg[: a.n_grad], a.exp_avg_sq[: a.n_grad], self.norm_out, lr,
                  self.betas[0], self.betas[1], self.eps, self.weight_decay, self.step_count, shadow)

    def zero_grad(self):
        self.arena.zero_grad()

    def state_dict(self):
        a = self.arena
        return {"step": self.step_count, "exp_avg": a.exp_avg.detach().cpu(), "exp_avg_sq": a.exp_avg_sq.detach().cpu(),
                "lr": self.param_groups[0]["lr"]}

    def load_state_dict(self, sd):
        self.step_count = int(sd["step"])
        self.arena.exp_avg.copy_(sd["exp_avg"])
        self.arena.exp_avg_sq.copy_(sd["exp_avg_sq"])
        self.param_groups[0]["lr"] = float(sd["lr"])


def cosine_with_warmup(base_lr, num_warmup_steps, num_training_steps, num_cycles=0.5):
    """transformers.get_cosine_schedule_with_warmup as a step -> lr function (trainer.py:137-155)"""

    def lr_at(step):
        if step < num_warmup_steps:
            return base_lr * float(step) / float(max(1, num_warmup_steps))
        progress = float(step - num_warmup_steps) / float(max(1, num_training_steps - num_warmup_steps))
        return base_lr * max(0.0, 0.5 * (1.0 + math.cos(math.pi * float(num_cycles) * 2.0 * progress)))

    return lr_at


class ArenaOptimizer(torch.optim.Optimizer):
    """The arena AdamW as a `torch.optim.Optimizer`, for Lightning's automatic optimization (the
    reference trains that way: trainer.py:117-177 returns torch AdamW, and best.yaml:105-106 puts
    gradient_clip_val: 1.0 and accumulate_grad_batches: 16 on the Trainer).

    * param_groups hold the trainable parameters; each `p.grad` is bound to the parameter's slice of
      the gradient arena (the HIP backward writes there, autograd never sets a .grad), so torch /
      Lightning code that walks `p.grad` -- GradScaler.unscale_ of precision=16, gradient-norm
      logging -- sees the real gradients;
    * zero_grad zeroes the arena and keeps the bindings (set_to_none is ignored: a None .grad would
      cut the view);
    * step(closure) runs the closure (Lightning's training_step + backward), then the fused clip +
      AdamW kernels over the whole arena with `max_grad_norm`, which
      SAM2LightningModule.configure_gradient_clipping sets from the Trainer's gradient_clip_val; with a
      process group of > 1 rank up (arena_ddp_strategy: no DistributedDataParallel wrapper) the arena
      was all-reduced before Lightning's GradScaler looked at it -- beside the staged backward by the
      graph-replayed micro-step, or by the module's backward hook (reduce_now) -- and the 1/world
      average is folded into the step's gradient scale;
    * the learning rate is param_groups[0]["lr"] (a torch LambdaLR drives it);
    * state_dict carries the arena moments (Lightning checkpoints)."""

    def __init__(self, arena, params, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01, max_grad_norm=0.0):
        params = list(params)
        super().__init__(params, dict(lr=float(lr), betas=tuple(betas), eps=float(eps),
                                      weight_decay=float(weight_decay)))
        self.impl = ArenaAdamW(arena, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                               max_grad_norm=max_grad_norm)
        self.arena = arena
        self.max_grad_norm = float(max_grad_norm or 0.0)
        self.reducer = None
        # set by SAM2LightningModule for the current accumulation window:
        self.hold_grads = False   # the next zero_grad keeps the arena (the graph-replayed micro-step filled it)
        self.window_scale = 1.0   # gradient scale of the window's arena (1/accumulate on the graph path)
        self.reduced = False      # the window's arena was already all-reduced (in the backward)
        self._bind()

    def _bind(self):
        for g in self.param_groups:
            for p in g["params"]:
                view = getattr(p, "_s2h_grad", None)
                if view is None:
                    raise ValueError("ArenaOptimizer: parameter without an arena gradient slice")
                if p.grad is None or p.grad.data_ptr() != view.data_ptr():
                    p.grad = view

    def zero_grad(self, set_to_none: bool = True):
        if self.hold_grads:  # Lightning's zero_grad after a graph-replayed first micro-batch: keep them
            self.hold_grads = False
        else:  # a new window (also after a step GradScaler skipped): fresh window state
            self.arena.zero_grad()
            self.reduced, self.window_scale = False, 1.0
        self._bind()

    @staticmethod
    def _world():
        import torch.distributed as dist
        return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1

    def reduce_now(self):
        """SUM all-reduce of the gradient arena over the process group (DDP without the wrapper,
        arena_ddp_strategy); called from the module's backward hook on a window's last micro-batch,
        i.e. before the precision plugin's GradScaler inspects the gradients"""
        if self._world() > 1 and not self.reduced:
            if self.reducer is None:
                from .ddp import ArenaGradReducer
                self.reducer = ArenaGradReducer(self.arena.grad_region())
            self.reducer.reduce()
        self.reduced = True

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        world = self._world()
        if world > 1 and not self.reduced:  # eager path without the module's backward hook
            self.reduce_now()
        scale = self.window_scale / world
        self.reduced, self.window_scale = False, 1.0
        self.impl.max_grad_norm = self.max_grad_norm
        self.impl.step(lr=self.param_groups[0]["lr"], grad_scale=scale)
        return loss

    def state_dict(self):
        sd = self.impl.state_dict()
        sd["param_groups_lr"] = [g["lr"] for g in self.param_groups]
        return sd

    def load_state_dict(self, sd):
        self.impl.load_state_dict(sd)
        for g, lr in zip(self.param_groups, sd.get("param_groups_lr", [])):
            g["lr"] = lr
