"""Parameter counting and freezing by module mapping (reference
sam2_video/utils/model_utils.py:9-77)."""
from __future__ import annotations

from typing import Any, Dict, List

import yaml
from torch import nn


def count_trainable_parameters(model: nn.Module) -> int:
    return sum(p.numel() for p in model.parameters() if p.requires_grad)


def count_total_parameters(model: nn.Module) -> int:
    return sum(p.numel() for p in model.parameters())


def get_model_info(model, checkpoint_path, config_path, device) -> Dict[str, Any]:
    t, n = count_trainable_parameters(model), count_total_parameters(model)
    return {"total_parameters": n, "trainable_parameters": t, "trainable_ratio": t / n if n else 0,
            "checkpoint_path": checkpoint_path, "config_path": config_path, "device": device}


def setup_trainable_modules(model, module_mapping: Dict[str, nn.Module], trainable_modules: List[str]) -> None:
    for name, module in module_mapping.items():
        if module is None:
            continue
        on = name in trainable_modules
        for p in module.parameters():
            p.requires_grad = on


def freeze_module_by_name(module_mapping, module_name):
    module = module_mapping.get(module_name)
    if module is None:
        raise KeyError(f"Module '{module_name}' not found")
    for p in module.parameters():
        p.requires_grad = False


def unfreeze_module_by_name(module_mapping, module_name):
    module = module_mapping.get(module_name)
    if module is None:
        raise KeyError(f"Module '{module_name}' not found")
    for p in module.parameters():
        p.requires_grad = True


def get_trainable_module_names(module_mapping) -> List[str]:
    return [n for n, m in module_mapping.items() if m is not None and any(p.requires_grad for p in m.parameters())]


def save_model_config(config_dict, path):
    with open(path, "w") as f:
        yaml.safe_dump(config_dict, f, default_flow_style=False)
