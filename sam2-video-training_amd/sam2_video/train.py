"""Training entry point for the reference's config tree (reference train.py:30-127) when Hydra,
Lightning and W&B are not installed:

    python -m sam2_video.train --config-dir /path/to/configs --config-name best \\
        trainer.max_steps=100 data.train_path=... [+key=value ...]
    python -m sam2_video.train --config-json composed.json [key=value ...]   # an already composed tree

Composes the config (sam2_video.utils.config.compose: defaults list, interpolation,
overrides), seeds, instantiates `module` and `data_module` with `_recursive_=False` and the
`trainer` section (resolving lightning.pytorch.trainer.trainer.Trainer to this build's
Trainer), runs `trainer.fit(module, data_module)` and writes a Lightning-layout checkpoint
(`model.`-prefixed state_dict) to <run_dir>/checkpoints/last.ckpt.  W&B logging, callbacks and
the post-training COCO inference (train.py:135-231) are out of scope.
"""
from __future__ import annotations

import argparse
import json
import os
import random
import sys

import torch


def main(argv=None, before_fit=None):
    """`before_fit(module, data_module, trainer)`, when given, runs right before trainer.fit (a test
    hook: e.g. the parity mode's dropout 0)"""
    ap = argparse.ArgumentParser()
    ap.add_argument("--config-dir", default="configs")
    ap.add_argument("--config-name", default="best")
    ap.add_argument("--config-json", default=None,
                    help="a config tree composed beforehand (JSON); overrides still apply")
    ap.add_argument("--run-dir", default=None)
    ap.add_argument("overrides", nargs="*")
    args = ap.parse_args(argv)
    from .model.build import instantiate
    from .utils.config import apply_overrides, compose

    run_dir = args.run_dir or os.path.join("outputs", args.config_name)
    if args.config_json:
        with open(args.config_json) as f:
            cfg = apply_overrides(json.load(f), args.overrides)
    else:
        cfg = compose(args.config_dir, args.config_name, args.overrides, run_dir=run_dir)
    seed = int(cfg.get("seed", 42))
    random.seed(seed)
    torch.manual_seed(seed)
    os.makedirs(run_dir, exist_ok=True)
    with open(os.path.join(run_dir, "config.json"), "w") as f:
        json.dump(cfg, f, indent=1, default=str)
    module = instantiate(cfg["module"], _recursive_=False)
    data_module = instantiate(cfg["data_module"], _recursive_=False)
    trainer = instantiate(cfg["trainer"])
    if before_fit is not None:
        before_fit(module, data_module, trainer)
    hist = trainer.fit(module, data_module)
    ck = os.path.join(run_dir, "checkpoints")
    os.makedirs(ck, exist_ok=True)
    trainer.save_checkpoint(os.path.join(ck, "last.ckpt"), module)
    for row in hist[-3:]:
        print(json.dumps(row), file=sys.stderr)
    return trainer


if __name__ == "__main__":
    main()
