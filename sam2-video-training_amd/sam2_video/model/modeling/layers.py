"""Parameter containers with the upstream SAM2 parameter names (state_dict
compatible: `<name>.weight` / `<name>.bias`).  They hold no compute of their
own: forward passes call sam2_video.kernels.functional, which reads the
compute-dtype weight from the arena (see kernels/arena.py)."""
from __future__ import annotations

import torch
from torch import nn

from ...kernels import functional as FN


def _compute(p):
    c = getattr(p, "_s2h_compute", None)
    if c is None:
        raise RuntimeError("parameters are not in a device arena yet: call SAM2Model.load(device) first")
    return c


class Linear(nn.Module):
    """nn.Linear-shaped parameters: weight [out, in], bias [out]."""

    def __init__(self, in_features, out_features, bias=True):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.weight = nn.Parameter(torch.zeros(out_features, in_features))
        self.bias = nn.Parameter(torch.zeros(out_features)) if bias else None

    def compute_weight(self):
        return _compute(self.weight).view(self.weight.shape[0], -1)

    def compute_bias(self):
        return self.bias.detach() if self.bias is not None else None

    def grad_views(self):
        return FN._grad_of(self.weight), FN._grad_of(self.bias)

    def forward(self, x, act=None, residual=None, drop_p=0.0):
        return FN.linear(x, self, act=act, residual=residual, drop_p=drop_p)


class FusedLinear:
    """Several Linear layers applied to the same input, run as one GEMM over their
    arena-adjacent weights (e.g. q/k/v projections).  Falls back to the members when
    the arena could not pack them."""

    def __init__(self, members, arena):
        self.members = list(members)
        self.arena = arena
        wn = [m.weight._s2h_name for m in self.members]
        bn = [m.bias._s2h_name for m in self.members]
        self.packed = arena.group_is_packed(wn) and arena.group_is_packed(bn)
        self.wn, self.bn = wn, bn
        self.weight = self.members[0].weight
        self.bias = self.members[0].bias
        self.out_features = sum(m.out_features for m in self.members)
        self.in_features = self.members[0].in_features

    def compute_weight(self):
        return self.arena.group_view(self.wn, "compute").view(self.out_features, self.in_features)

    def compute_bias(self):
        return self.arena.group_view(self.bn, "data")

    def grad_views(self):
        if FN._grad_of(self.weight) is None:
            return None, None
        return (self.arena.group_view(self.wn, "grad").view(self.out_features, self.in_features),
                self.arena.group_view(self.bn, "grad"))

    def __call__(self, x, act=None, residual=None, drop_p=0.0, rope=None):
        if self.packed:
            return FN.linear(x, self, act=act, residual=residual, drop_p=drop_p, rope=rope)
        return None


class Conv2d(Linear):
    """nn.Conv2d parameters (weight [co, ci, k, k]) used as an NHWC GEMM: 1x1 directly,
    k > 1 through im2col (column order (ci, ky, kx) = the weight's own layout)."""

    def __init__(self, in_ch, out_ch, kernel_size=1, stride=1, padding=0, groups=1):
        nn.Module.__init__(self)
        self.in_ch, self.out_ch, self.k, self.stride, self.padding = in_ch, out_ch, kernel_size, stride, padding
        self.groups = groups
        self.weight = nn.Parameter(torch.zeros(out_ch, in_ch // groups, kernel_size, kernel_size))
        self.bias = nn.Parameter(torch.zeros(out_ch))


class ConvTranspose2x2(nn.Module):
    """nn.ConvTranspose2d(k=2, s=2) parameters: weight [ci, co, 2, 2], bias [co]."""

    def __init__(self, in_ch, out_ch):
        super().__init__()
        self.in_ch, self.out_ch = in_ch, out_ch
        self.weight = nn.Parameter(torch.zeros(in_ch, out_ch, 2, 2))
        self.bias = nn.Parameter(torch.zeros(out_ch))

    def compute_weight(self):
        return _compute(self.weight).view(self.in_ch, self.out_ch * 4)


class LayerNorm(nn.Module):
    """nn.LayerNorm / LayerNorm2d parameters (weight, bias) + eps."""

    def __init__(self, dim, eps=1e-5):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(dim))
        self.bias = nn.Parameter(torch.zeros(dim))

    def forward(self, x):
        return FN.layer_norm(x, self, self.eps)


class LayerNorm2d(LayerNorm):
    """sam2_utils.py:141-153 -- channel norm; feature maps are NHWC here, so a row norm."""

    def __init__(self, dim, eps=1e-6):
        super().__init__(dim, eps)


class Embedding(nn.Module):
    def __init__(self, num, dim):
        super().__init__()
        self.weight = nn.Parameter(torch.zeros(num, dim))

    def compute_weight(self):
        return _compute(self.weight)


class MLP(nn.Module):
    """sam2_utils.py:112-136 (activation relu/gelu, optional sigmoid output)"""

    def __init__(self, input_dim, hidden_dim, output_dim, num_layers, activation="relu", sigmoid_output=False):
        super().__init__()
        self.num_layers = num_layers
        h = [hidden_dim] * (num_layers - 1)
        self.layers = nn.ModuleList(Linear(n, k) for n, k in zip([input_dim] + h, h + [output_dim]))
        self.act = activation
        self.sigmoid_output = sigmoid_output

    def forward(self, x, residual=None, norm=None):
        """norm: the output (+ residual) LayerNorm'ed -- with a residual, the last layer, the add and the
        LayerNorm as one launch (FN.linear_add_layer_norm; the two-way block's MLP -> norm3)"""
        for i, layer in enumerate(self.layers):
            last = i == self.num_layers - 1
            if last:
                if norm is not None and residual is not None and not self.sigmoid_output and \
                        FN._linear_ln_ok(x, layer, norm):
                    return FN.linear_add_layer_norm(x, layer, residual, norm, norm.eps)[0]
                x = layer(x, act="sigmoid" if self.sigmoid_output else None, residual=residual)
            else:
                x = layer(x, act=self.act)
        return norm(x) if norm is not None else x


class Identity(nn.Module):
    """index placeholder (activation slots of nn.Sequential in the upstream modules)"""

    def forward(self, x):
        return x


def param_compute(p):
    return _compute(p)
