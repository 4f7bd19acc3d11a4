"""Flat parameter arena: one contiguous fp32 master buffer for every parameter,
one contiguous fp32 gradient buffer (and AdamW moments) for the parameters that
receive gradients, and a bf16 shadow copy used by the bf16 compute path.

  * nn.Parameter objects keep their names/shapes (state_dict compatible); their
    `.data` becomes a view into the arena.
  * `p._s2h_grad`  -> fp32 view into the gradient arena (backward kernels
    accumulate into it directly; torch's .grad is never used).
  * `p._s2h_compute` -> view of the weight in the compute dtype (bf16 shadow or
    the fp32 master itself).
  * `groups`: lists of parameter names that must be adjacent (in order) so the
    kernels can treat them as one matrix -- e.g. q/k/v projection weights of a
    self-attention fused into a single [3*C, C] GEMM operand.

The gradient region is one contiguous range, so clip-norm, AdamW and the DDP
all-reduce each run as a single kernel / collective over it.
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Sequence

import torch

from . import ops

ALIGN = 64  # elements: keeps every view 16-B aligned for both fp32 and bf16 vector loads


def _align(n):
    return (n + ALIGN - 1) // ALIGN * ALIGN


class ParamArena:
    def __init__(self, named_params: Sequence, grad_names: Iterable[str], compute_dtype, device,
                 groups: Sequence[Sequence[str]] = (), tail_prefixes: Sequence[str] = (), tail_rank=None):
        """tail_prefixes: gradient-receiving parameters under these name prefixes go to the END of
        the gradient region (their gradients are completed last in the backward -- the image
        encoder's -- so the rest of the region can be all-reduced while they are computed);
        `grad_split` is the offset where they start.  tail_rank (name -> int or None) instead puts
        the ranked gradient-receiving parameters at the end in rank order (the order the staged
        backward completes them); `grad_cuts` = [start of each rank's range ..., n_grad]."""
        grad_names = set(grad_names)
        params = dict(named_params)
        tail = tuple(tail_prefixes)
        ranks = {}
        if tail_rank is not None:
            ranks = {n: tail_rank(n) for n, _ in named_params if n in grad_names}
            ranks = {n: r for n, r in ranks.items() if r is not None}
            head = [(n, p) for n, p in named_params if n not in ranks]
            tailp = sorted([(n, p) for n, p in named_params if n in ranks], key=lambda np_: ranks[np_[0]])
            named_params = head + tailp
            tail = tuple(ranks)  # exact names (str.startswith accepts a tuple)
        elif tail:  # stable partition of the gradient-receiving names: tail prefixes last
            named_params = ([(n, p) for n, p in named_params if not (n in grad_names and n.startswith(tail))]
                            + [(n, p) for n, p in named_params if n in grad_names and n.startswith(tail)])
        order: List[str] = []
        seen = set()
        # grad-receiving params first (contiguous gradient region), grouped names kept adjacent
        grouped = {n: g for g in groups for n in g}
        for want_grad in (True, False):
            for n, _ in named_params:
                if n in seen or ((n in grad_names) != want_grad):
                    continue
                block = grouped.get(n, [n])
                if any(((m in grad_names) != want_grad) for m in block):
                    block = [n]  # mixed trainability: group cannot be honoured
                for m in block:
                    if m not in seen and m in params:
                        order.append(m)
                        seen.add(m)
        self.order = order
        self.offsets: Dict[str, int] = {}
        off = 0
        n_grad = 0
        self.grad_names = [n for n in order if n in grad_names]
        for n in order:
            numel = params[n].numel()
            # grouped members are packed without padding so they form one matrix
            self.offsets[n] = off
            nxt = order[order.index(n) + 1] if order.index(n) + 1 < len(order) else None
            packed = nxt is not None and grouped.get(n) is not None and nxt in grouped.get(n)
            off += numel if (packed and numel % ALIGN == 0) else _align(numel)
            if n in grad_names:
                n_grad = off
        self.total = _align(off)
        self.n_grad = _align(n_grad)
        if ranks:
            tails = [self.offsets[n] for n in order if n in ranks]
        else:
            tails = [self.offsets[n] for n in order if n in grad_names and tail and n.startswith(tail)]
        self.grad_split = min(tails) if tails else self.n_grad
        # start offset of every rank's range (empty ranks start where the next one does) + n_grad
        self.grad_cuts = [self.grad_split, self.n_grad]
        if ranks:
            top = max(ranks.values())
            starts = {}
            for n in order:
                if n in ranks:
                    starts.setdefault(ranks[n], self.offsets[n])
            cuts = [self.n_grad] * (top + 2)
            for r in range(top, -1, -1):
                cuts[r] = starts.get(r, cuts[r + 1])
            self.grad_cuts = cuts
        self.device = device
        self.compute_dtype = compute_dtype
        self.data = torch.zeros(self.total, dtype=torch.float32, device=device)
        self.grad = torch.zeros(max(self.n_grad, 1), dtype=torch.float32, device=device)
        self.exp_avg = torch.zeros_like(self.grad)
        self.exp_avg_sq = torch.zeros_like(self.grad)
        self.shadow = (torch.zeros(self.total, dtype=torch.bfloat16, device=device)
                       if compute_dtype == torch.bfloat16 else None)
        self.params = params
        for n in order:
            p = params[n]
            o = self.offsets[n]
            view = self.data[o:o + p.numel()].view(p.shape)
            view.copy_(p.data.to(device=device, dtype=torch.float32))
            p.data = view
            p._s2h_name = n
            p._s2h_grad = self.grad[o:o + p.numel()].view(p.shape) if n in grad_names else None
            if self.shadow is not None:
                p._s2h_compute = self.shadow[o:o + p.numel()].view(p.shape)
            else:
                p._s2h_compute = view
        self.refresh_shadow()

    # contiguous multi-parameter views (valid for a group declared at construction)
    def group_view(self, names: Sequence[str], which="compute"):
        o0 = self.offsets[names[0]]
        n = sum(self.params[m].numel() for m in names)
        for a, b in zip(names, names[1:]):
            assert self.offsets[b] == self.offsets[a] + self.params[a].numel(), "group not packed"
        if which == "compute":
            buf = self.shadow if self.shadow is not None else self.data
        elif which == "grad":
            buf = self.grad
        else:
            buf = self.data
        return buf[o0:o0 + n]

    def group_is_packed(self, names: Sequence[str]) -> bool:
        try:
            for a, b in zip(names, names[1:]):
                if self.offsets[b] != self.offsets[a] + self.params[a].numel():
                    return False
            g = [m in self.grad_names for m in names]
            return all(g) or not any(g)
        except KeyError:
            return False

    def refresh_shadow(self):
        if self.shadow is not None:
            ops.cast(self.data, torch.bfloat16, out=self.shadow)

    def zero_grad(self):
        self.grad.zero_()

    def grad_region(self):
        return self.grad[: self.n_grad]
