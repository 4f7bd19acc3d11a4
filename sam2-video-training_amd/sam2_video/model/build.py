"""`_target_` resolver: the reference's model YAML instantiates upstream
`sam2.modeling.*` classes (configs/sam2/sam2.1_hiera_t.yaml:5-85); upstream sam2
is not a dependency here, so those class paths resolve to this build's modules.
Accepts a YAML path (reference layout: top-level `model:` key) or a named size
("tiny" | "small" | "base_plus" | "large", optionally "@<image_size>").
"""
from __future__ import annotations

import importlib
import os

import yaml

from . import configs

_TARGETS = {
    "sam2.modeling.sam2_base.SAM2Base": "sam2_video.model.modeling.sam2_base.SAM2Base",
    "sam2.modeling.backbones.image_encoder.ImageEncoder":
        "sam2_video.model.modeling.backbones.image_encoder.ImageEncoder",
    "sam2.modeling.backbones.image_encoder.FpnNeck": "sam2_video.model.modeling.backbones.image_encoder.FpnNeck",
    "sam2.modeling.backbones.hieradet.Hiera": "sam2_video.model.modeling.backbones.hieradet.Hiera",
    "sam2.modeling.position_encoding.PositionEmbeddingSine":
        "sam2_video.model.modeling.position_encoding.PositionEmbeddingSine",
    "sam2.modeling.memory_attention.MemoryAttention": "sam2_video.model.modeling.memory_attention.MemoryAttention",
    "sam2.modeling.memory_attention.MemoryAttentionLayer":
        "sam2_video.model.modeling.memory_attention.MemoryAttentionLayer",
    "sam2.modeling.sam.transformer.RoPEAttention": "sam2_video.model.modeling.sam.transformer.RoPEAttention",
    "sam2.modeling.memory_encoder.MemoryEncoder": "sam2_video.model.modeling.memory_encoder.MemoryEncoder",
    "sam2.modeling.memory_encoder.MaskDownSampler": "sam2_video.model.modeling.memory_encoder.MaskDownSampler",
    "sam2.modeling.memory_encoder.Fuser": "sam2_video.model.modeling.memory_encoder.Fuser",
    "sam2.modeling.memory_encoder.CXBlock": "sam2_video.model.modeling.memory_encoder.CXBlock",
}


# Lightning classes of the reference configs (best.yaml:13,22,99); Lightning is not installed here, so the
# trainer resolves to this build's Lightning-API Trainer (training/trainer.py) unless it is importable
_LIGHTNING = {
    "lightning.pytorch.trainer.trainer.Trainer": "sam2_video.training.trainer.Trainer",
    "lightning.pytorch.Trainer": "sam2_video.training.trainer.Trainer",
    "lightning.Trainer": "sam2_video.training.trainer.Trainer",
}


def _resolve(target: str):
    path = _TARGETS.get(target, target)
    if path in _LIGHTNING:
        try:
            importlib.import_module("lightning")
        except ImportError:
            path = _LIGHTNING[path]
    mod, name = path.rsplit(".", 1)
    return getattr(importlib.import_module(mod), name)


def _coerce(v):
    if isinstance(v, str):
        try:
            return float(v) if any(c in v for c in ".eE") else int(v)
        except ValueError:
            return v
    return v


def instantiate(cfg, _recursive_: bool = True, **override):
    """hydra.utils.instantiate for `_target_` dicts; `_recursive_=False` passes nested sections
    through as plain dicts (train.py:103-104 instantiates module / data_module that way)."""
    if isinstance(cfg, dict):
        if "_target_" in cfg:
            rec = cfg.get("_recursive_", _recursive_)
            kw = {k: (instantiate(v) if rec else v) for k, v in cfg.items() if k not in ("_target_", "_recursive_")}
            kw.update(override)
            return _resolve(cfg["_target_"])(**kw)
        return {k: instantiate(v) for k, v in cfg.items()}
    if isinstance(cfg, list):
        return [instantiate(v) for v in cfg]
    return _coerce(cfg)


def load_model_config(config_path: str, image_size=None) -> dict:
    """named size or YAML file -> `_target_` dict of the SAM2Base model"""
    name, _, sz = str(config_path).partition("@")
    key = configs.ALIASES.get(name, name)
    if key in configs.TRUNKS:
        return configs.model_config(key, int(image_size or sz or 512))
    path = config_path
    if not os.path.isabs(path) and not os.path.exists(path):
        here = os.path.join(os.path.dirname(__file__), "..", "configs", path)
        path = here if os.path.exists(here) else path
    if not os.path.exists(path):
        # upstream config names as the reference YAMLs spell them (best.yaml:32
        # `config_path: sam2/sam2.1_hiera_t.yaml`): resolve to the built-in table
        stem = os.path.basename(name)
        stem = stem[:-5] if stem.endswith(".yaml") else stem
        for prefix in ("sam2.1_", "sam2_"):
            if stem.startswith(prefix):
                stem = stem[len(prefix):]
        key = configs.ALIASES.get(stem, stem)
        if key in configs.TRUNKS:
            # the reference's own configs/sam2/sam2.1_hiera_t.yaml sets image_size 384 (:88);
            # upstream SAM2.1 configs use 1024
            default = 384 if (name.startswith("sam2/") and key == "tiny") else 1024
            return configs.model_config(key, int(image_size or sz or default))
    with open(path) as f:
        y = yaml.safe_load(f)
    cfg = y.get("model", y)
    if image_size:
        cfg["image_size"] = int(image_size)
    return cfg
