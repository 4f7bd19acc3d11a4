"""bf16 bench-path gradients against the reference's fp32 and CPU-bf16 steps (B+ 256^2, 8 frames):
per-tensor relative error of ours and of the reference's bf16 run, grouped by module, for the
current environment switches (S2H_VFOLD, S2H_ATTN_CFG, ...).  GPU only.

    python tools/bf16_grad_diag.py --tag default > gpurun_out/diag_default.json"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="default")
    ap.add_argument("--case", default="t8", choices=["t8", "t4"])
    ap.add_argument("--dtype", default="bf16")
    args = ap.parse_args()
    import torch
    from step_harness import ALL, bf16_grad_report, build_model, golden_batch, grads_by_name, load_golden
    from test_training_step_gpu import loss_section, make_module, step
    if args.case == "t8":
        gf, gb = load_golden("bplus256_point_all_t8"), load_golden("bplus256_point_all_t8_bf16")
    else:
        gf, gb = load_golden("bplus256_point_all"), load_golden("bplus256_point_all_bf16")
    model = build_model("base_plus", 256, ALL, "point", dtype=args.dtype, seed=int(gf["meta/seed"]))
    mod = make_module(model, loss_section(gf))
    total = step(mod, golden_batch(gf).to("cuda"))
    grads = grads_by_name(model)
    rows, bad = bf16_grad_report(grads, gf, gb)
    ratio = {k[6:]: (float(grads[k[6:]].double().norm()) / max(float(gf[k]), 1e-30), float(gb[k]) / max(float(gf[k]), 1e-30))
             for k in gf if k.startswith("gnorm/")}
    out = {"tag": args.tag, "env": {k: v for k, v in os.environ.items() if k.startswith("S2H_")},
           "loss": float(total), "loss_ref32": float(gf["loss/total_loss"]), "n_bad": len(bad),
           "bad": bad[:40], "rows": rows, "norm_ratio": ratio}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
