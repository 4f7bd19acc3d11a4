"""MX-fp8 drift against the fp32 and bf16 modes of this build on one B+ 256^2 clip (dropout off),
per fp8 layer set: which projections / FFN take the MX-fp8 path changes the forward error.
  python tools/fp8_drift.py      (GPU box)"""
import sys

import torch

sys.path.insert(0, "tests"); sys.path.insert(0, "."); sys.path.insert(0, "sam2-video-training_amd")
from step_harness import ALL, build_model, mask_iou, run_step  # noqa: E402
from test_configs_gpu import _clips  # noqa: E402

from sam2_video.kernels import fp8  # noqa: E402

clip = _clips([31], 4, 256, 4, 4)[0]
SETS = {"all": fp8.FP8_PREFIXES, "trunk": ("image_encoder.trunk.",), "memattn": ("memory_attention.",),
        "twoway": ("sam_mask_decoder.transformer.",), "trunk_mlp": ("image_encoder.trunk.blocks.",)}
res = {}
for name, dt in [("fp32", "fp32"), ("bf16", "bf16")] + [(k, "fp8") for k in SETS]:
    if dt == "fp8":
        fp8.FP8_PREFIXES = SETS[name]
    m = build_model("base_plus", 256, ALL, dtype=dt, dropout=0.0)
    if name == "trunk_mlp":  # only the MLPs of the trunk blocks
        for n, mod in m.named_modules():
            if getattr(mod, "_s2h_fp8", False) and ".mlp." not in n:
                mod._s2h_fp8 = False
    stages, merged, losses, _ = run_step(m, clip)
    res[name] = ([s["pred_masks"].detach().float().cpu() for s in stages], float(losses["total_loss"].detach()),
                 m.arena.grad_region().detach().float().clone())
    del m, stages, merged
    torch.cuda.empty_cache()
ref = res["fp32"]
for name in ["bf16"] + list(SETS):
    r = res[name]
    ious = [round(mask_iou(a, b), 4) for a, b in zip(ref[0], r[0])]
    cos = float((ref[2] * r[2]).sum() / (ref[2].norm() * r[2].norm()))
    print(f"{name:10s} vs fp32: IoU {ious} loss {ref[1]:.4f} -> {r[1]:.4f} grad cos {cos:.4f}")
