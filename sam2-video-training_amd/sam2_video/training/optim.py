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
