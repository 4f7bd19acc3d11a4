"""Deterministic synthetic weights keyed by state_dict name (no checkpoints exist
offline).  The same function seeds the golden-fixture generator (which loads
this file by path into the reference model) and this build's model, so parity
runs never ship weight files.  Depends on torch only.
"""
from __future__ import annotations

import math
import zlib

import torch


def _gen(name: str, seed: int) -> torch.Generator:
    return torch.Generator().manual_seed((zlib.crc32(name.encode()) ^ (seed * 0x9E3779B1)) & 0x7FFFFFFF)


def synth_tensor(name: str, shape, seed: int = 0) -> torch.Tensor:
    shape = tuple(int(s) for s in shape)
    g = _gen(name, seed)
    z = torch.randn(shape, generator=g, dtype=torch.float32) if len(shape) else torch.randn((), generator=g)
    leaf = name.rsplit(".", 1)[-1]
    if name.endswith("positional_encoding_gaussian_matrix"):
        return z  # PositionEmbeddingRandom(scale=1) buffer
    if "pred_obj_score_head" in name and leaf == "bias" and shape == (1,):
        return torch.full(shape, 2.0)  # object present -> masks not gated to NO_OBJ_SCORE
    if leaf == "gamma":  # CXBlock layer scale
        return 0.1 + 0.02 * z
    if len(shape) >= 2 and leaf == "weight":
        fan_in = math.prod(shape[1:])
        return z / math.sqrt(max(fan_in, 1))
    if leaf == "weight" and len(shape) == 1:  # LayerNorm / LayerNorm2d scale
        return 1.0 + 0.1 * z
    if leaf == "bias":
        return 0.02 * z
    return 0.02 * z  # pos embeds, tokens, tpos encodings, no-object embeddings


def synth_state_dict(named_shapes, seed: int = 0):
    """named_shapes: iterable of (name, shape) -> {name: tensor}"""
    return {n: synth_tensor(n, s, seed) for n, s in named_shapes}
