"""Hydra-style config composition for the reference's configs/ tree, without Hydra (not
installed here): the defaults list (`- config`, `- data: cholecseg8k`, `- _self_`), deep
merge, `${a.b}` interpolation (`${hydra:run.dir}` -> the run directory) and `key=value` /
`+key=value` command-line overrides, as `python train.py --config-name best key=val` uses them
(reference train.py:30-32, README.md:104-121)."""
from __future__ import annotations

import copy
import os
import re
from typing import Any, Dict, List, Optional

import yaml

_INTERP = re.compile(r"\$\{([^}]+)\}")


def _load(path: str) -> Dict[str, Any]:
    with open(path) as f:
        return yaml.safe_load(f) or {}


def merge(base: Dict[str, Any], over: Dict[str, Any]) -> Dict[str, Any]:
    """deep merge (dicts merge key by key, everything else is replaced)"""
    out = copy.deepcopy(base)
    for k, v in (over or {}).items():
        if isinstance(v, dict) and isinstance(out.get(k), dict):
            out[k] = merge(out[k], v)
        else:
            out[k] = copy.deepcopy(v)
    return out


def _compose_file(config_dir: str, name: str) -> Dict[str, Any]:
    name = name[:-5] if name.endswith(".yaml") else name
    raw = _load(os.path.join(config_dir, name + ".yaml"))
    defaults = raw.pop("defaults", None) or ["_self_"]
    if "_self_" not in defaults:
        defaults = list(defaults) + ["_self_"]
    out: Dict[str, Any] = {}
    for d in defaults:
        if d == "_self_":
            out = merge(out, raw)
        elif isinstance(d, str):
            out = merge(out, _compose_file(config_dir, d))
        elif isinstance(d, dict):
            for group, opt in d.items():
                if opt is None:
                    continue
                group = group.lstrip("+")
                sub = _compose_file(os.path.join(config_dir, group), str(opt))
                out = merge(out, {group: sub})
    return out


def _get_path(cfg, path):
    cur = cfg
    for part in path.split("."):
        if not isinstance(cur, dict) or part not in cur:
            raise KeyError(f"interpolation ${{{path}}}: '{part}' not found")
        cur = cur[part]
    return cur


def _resolve(node, root, run_dir, depth=0):
    if depth > 32:
        raise ValueError("interpolation cycle")
    if isinstance(node, dict):
        return {k: _resolve(v, root, run_dir, depth) for k, v in node.items()}
    if isinstance(node, list):
        return [_resolve(v, root, run_dir, depth) for v in node]
    if not isinstance(node, str) or "${" not in node:
        return node

    def one(expr):
        if expr.startswith("hydra:"):
            key = expr[len("hydra:"):]
            return run_dir if key in ("run.dir", "runtime.output_dir") else os.path.join(run_dir, key)
        return _resolve(_get_path(root, expr), root, run_dir, depth + 1)

    m = _INTERP.fullmatch(node.strip())
    if m:  # the whole value is one interpolation: keep its type (dicts, lists, numbers)
        return one(m.group(1))
    return _INTERP.sub(lambda mm: str(one(mm.group(1))), node)


def _set_path(cfg, path, value, add=False):
    parts = path.split(".")
    cur = cfg
    for p in parts[:-1]:
        if p not in cur or not isinstance(cur[p], dict):
            if not add and p not in cur:
                raise KeyError(f"override {path}: '{p}' not in config (use +{path}=...)")
            cur[p] = {}
        cur = cur[p]
    if not add and parts[-1] not in cur:
        raise KeyError(f"override {path}: key not in config (use +{path}=...)")
    cur[parts[-1]] = value


def apply_overrides(cfg: Dict[str, Any], overrides: List[str]) -> Dict[str, Any]:
    cfg = copy.deepcopy(cfg)
    for ov in overrides or []:
        key, _, val = ov.partition("=")
        add = key.startswith("+")
        key = key.lstrip("+")
        value = yaml.safe_load(val) if val != "" else None
        _set_path(cfg, key, value, add=add)
    return cfg


def compose(config_dir: str, config_name: str, overrides: Optional[List[str]] = None,
            run_dir: str = "outputs/run") -> Dict[str, Any]:
    """configs/<config_name>.yaml with its defaults list, overrides, interpolations resolved"""
    cfg = _compose_file(config_dir, config_name)
    cfg = apply_overrides(cfg, overrides or [])
    return _resolve(cfg, cfg, run_dir)
