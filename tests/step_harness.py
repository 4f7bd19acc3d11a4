"""Shared helpers: run one training step of the HIP build on the GPU and compare it
with golden fixtures from the reference / with the CPU oracle (tests only)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
ALL = ["image_encoder", "memory_attention", "memory_encoder", "mask_decoder", "prompt_encoder"]
CASES = {
    "tiny256_point_all": ("tiny", "point", ALL),
    "tiny256_point_mem": ("tiny", "point", ["memory_attention", "memory_encoder"]),
    "tiny256_box_all": ("tiny", "box", ALL),
    "bplus128_point_all": ("base_plus", "point", ALL),
    "bplus128_point_all_t8": ("base_plus", "point", ALL),
    "tiny256_point_all_multi": ("tiny", "point", ALL),
    "tiny256_mask_all": ("tiny", "mask", ALL),
    "bplus256_point_all": ("base_plus", "point", ALL),
    # Hiera-L trunk (BASELINE config 4's model): stages [2, 6, 36, 4], head dim 72
    "large128_point_all": ("large", "point", ALL),
}
# reference steps under CPU bf16 autocast (oracle/gen_golden.py), with their fp32 twin
BF16_CASES = {"bplus256_point_all_bf16": "bplus256_point_all"}


def load_golden(name):
    return torch.load(os.path.join(GOLD, name + ".pt"), weights_only=True)


def build_model(size, image_size, trainable, prompt="point", dtype="fp32", seed=0, dropout=0.0):
    from sam2_video.model.sam2model import SAM2Model
    m = SAM2Model(None, f"{size}@{image_size}", trainable_modules=trainable, prompt_type=prompt, compute_dtype=dtype,
                  init_seed=seed)
    m.load("cuda")
    m.train()
    m.set_dropout(dropout)
    return m


def run_step(model, batch, criterion=None):
    """forward (keeping per-object outputs) + loss + backward; returns (stages, merged, losses)"""
    from sam2_video.model.losses import MultiStepMultiMasksAndIous
    from sam2_video.utils.masks import merge_object_results_to_category
    if criterion is None:
        criterion = MultiStepMultiMasksAndIous({"loss_mask": 20, "loss_dice": 1, "loss_iou": 1, "loss_class": 0},
                                               supervise_all_iou=True, iou_use_l1_loss=True)
    model.arena.zero_grad()
    bo = model.forward_image(batch.flat_img_batch)
    bo = model.prepare_prompt_inputs(bo, batch)
    stages = model.forward_tracking(bo, batch)
    merged = merge_object_results_to_category(stages, bo["obj_to_cat"], bo["num_categories"])
    losses = criterion(merged, batch.masks)
    losses["total_loss"].backward()
    torch.cuda.synchronize()
    return stages, merged, losses, bo


def golden_batch(g):
    from sam2_video.data.synthetic import synthetic_batch
    T, S = int(g["meta/T"]), int(g["meta/image_size"])
    n_cat = g["in/masks_count"].shape[1]
    n_obj = int((g["in/masks_count"][0] > 0).sum())
    parts = g["meta/parts"].tolist() if "meta/parts" in g else None
    return synthetic_batch(int(g["meta/clip_idx"]), T, S, n_cat, n_obj, parts)


def grads_by_name(model):
    out = {}
    for n, p in model.named_parameters():
        gv = getattr(p, "_s2h_grad", None)
        if gv is not None:
            out[n] = gv.detach().float().cpu()
    return out


def structural_zero_grads(gf):
    """key biases of attentions without RoPE: their gradient is exactly zero in exact arithmetic
    (softmax is shift invariant along the keys), the reference holds fp32 cancellation noise
    there (|dk_bias| ~ 1e-8 x |dk_weight|)"""
    out = set()
    for k in [k for k in gf if k.startswith("gnorm/") and k.endswith("k_proj.bias")]:
        n = k[6:]
        if float(gf[k]) <= 1e-6 * float(gf["gnorm/" + n[:-4] + "weight"]):
            out.add(n)
    return out


def grad_group(name):
    """module group of a parameter for the bf16 gradient statistics (the decoder split by block)"""
    parts = name.split(".")
    return ".".join(parts[:2]) if parts[0] == "sam_mask_decoder" else parts[0]


def bf16_grad_report(grads, gf, gb, floor=0.01, eps_cos=0.002):
    """the bench path's (bf16) gradients against the reference's fp32 step (gf), with the
    reference's own CPU-bf16-autocast step (gb) of the same clip as the scale.

    Relative error of an entry: | |g| - |g32| | / |g32| for `gnorm/` entries, |g - g32| / |g32|
    (Frobenius) for `grad/` tensors; e_ours for this build, e_ref for the reference's bf16 step.
    Where the whole tensor is stored (`grad/`), the gnorm entry's e_ref is the reference's VECTOR
    drift |g16 - g32| / |g32| (it bounds what the norm can be off by; the norm of a noise-dominated
    vector can land near |g32| by chance -- the decoder's image -> token q bias: norm 6 % off in the
    reference's bf16 run, the vector 32 %).  Bounds, per module group (`grad_group`) and kind:
      * groups of >= 8 entries: RMS of e_ours <= 1.25 RMS of e_ref + floor;
      * every entry: e_ours <= 2 max(e_ref, q90) + floor, q90 = the 90th percentile of e_ref in
        its group (a bf16 gradient's drift is noisy per tensor -- the reference's own bf16 run puts
        one q projection 0.5 % and the next 5 % off -- so a tensor is held to twice what the
        reference's bf16 step shows on that tensor or on the group's worse tensors);
      * every non-zero `grad/` tensor: 1 - cos(g, g32) <= 2 (1 - cos(g16, g32)) + eps_cos.
    Structural zeros (`structural_zero_grads`): |g| <= 2 |g16| + 1e-3 |sibling weight grad|.
    Returns (rows, bad); rows = (name, kind, e_ours, e_ref[, cos_ours, cos_ref])."""
    import collections
    import math
    structural = structural_zero_grads(gf)
    rows, bad = [], []
    for k in gf:
        if not (k.startswith("gnorm/") or k.startswith("grad/")):
            continue
        kind, n = k.split("/", 1)
        g = grads[n].double()
        if n in structural:
            if kind == "gnorm":
                sib = float(gf["gnorm/" + n[:-4] + "weight"])
                if float(g.norm()) > 2.0 * float(gb[k]) + 1e-3 * sib:
                    bad.append((n, "structural", float(g.norm()), float(gb[k]), sib))
            continue
        if kind == "gnorm":
            r32, r16, got = float(gf[k]), float(gb[k]), float(g.norm())
            e_ref = abs(r16 - r32)
            if "grad/" + n in gf:
                e_ref = max(e_ref, float((gb["grad/" + n].double() - gf["grad/" + n].double()).norm()))
            rows.append((n, "gnorm", abs(got - r32) / max(r32, 1e-30), e_ref / max(r32, 1e-30)))
        else:
            r32, r16 = gf[k].double(), gb[k].double()
            n32, n16, no = float(r32.norm()), float(r16.norm()), float(g.norm())
            e_ours, e_ref = float((g - r32).norm()), float((r16 - r32).norm())
            if n32 == 0.0:  # an unused embedding row set: both must stay zero
                if no != 0.0:
                    bad.append((n, "zero", no, n16))
                continue
            c_ours = float((g.flatten() @ r32.flatten()) / max(no * n32, 1e-300))
            c_ref = float((r16.flatten() @ r32.flatten()) / max(n16 * n32, 1e-300))
            rows.append((n, "grad", e_ours / n32, e_ref / n32, c_ours, c_ref))
            if 1.0 - c_ours > 2.0 * (1.0 - c_ref) + eps_cos:
                bad.append(rows[-1] + ("cos",))
    groups = collections.defaultdict(list)
    for r in rows:
        groups[(grad_group(r[0]), r[1])].append(r)
    for key, rs in groups.items():
        ref = sorted(r[3] for r in rs)
        q90 = ref[min(len(ref) - 1, int(0.9 * len(ref)))]
        rms_o = math.sqrt(sum(r[2] ** 2 for r in rs) / len(rs))
        rms_r = math.sqrt(sum(r[3] ** 2 for r in rs) / len(rs))
        if len(rs) >= 8 and rms_o > 1.25 * rms_r + floor:
            bad.append((key, "rms", rms_o, rms_r))
        for r in rs:
            if r[2] > 2.0 * max(r[3], q90) + floor:
                bad.append(r + ("q90", q90))
    return rows, bad


def mask_iou(a, b):
    a, b = a > 0, b > 0
    inter = (a & b).sum().item()
    uni = (a | b).sum().item()
    return inter / max(uni, 1)
