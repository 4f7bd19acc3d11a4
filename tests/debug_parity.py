"""Diagnostic (not a test): prints per-stage parity numbers of the HIP step vs golden.
python tests/debug_parity.py [case] [fp32|bf16]"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "sam2-video-training_amd"))
import torch  # noqa: E402

from step_harness import CASES, build_model, golden_batch, grads_by_name, load_golden, mask_iou, run_step  # noqa

name = sys.argv[1] if len(sys.argv) > 1 else "tiny256_point_all"
dt = sys.argv[2] if len(sys.argv) > 2 else "fp32"
g = load_golden(name)
size, prompt, trainable = CASES[name]
model = build_model(size, int(g["meta/image_size"]), trainable, prompt, dtype=dt, seed=int(g["meta/seed"]))
batch = golden_batch(g).to("cuda")
t0 = time.time()
stages, merged, losses, bo = run_step(model, batch)
print(f"step {time.time() - t0:.2f}s obj_to_cat {bo['obj_to_cat']} ref {g['obj_to_cat'].tolist()}")
fpn_last = bo["backbone_fpn"][-1].detach().float().cpu()
ref = g["feat/fpn_last"]  # [T, C, h, w]
print("fpn_last maxdiff", (fpn_last.permute(0, 3, 1, 2) - ref).abs().max().item(), "scale", ref.abs().max().item())
for t, st in enumerate(stages):
    got = st["pred_masks"].detach().float().cpu()
    r = g[f"obj/{t}/low_res"]
    print(f"frame {t}: lowres maxdiff {(got - r).abs().max().item():.3e} (scale {r.abs().max().item():.2f}) "
          f"iou {mask_iou(got, r):.5f} ious {st['multistep_pred_ious'][0].detach().cpu().view(-1).tolist()} "
          f"ref {g[f'obj/{t}/ious'].view(-1).tolist()} score {st['multistep_object_score_logits'][0].view(-1).tolist()}"
          f" ref {g[f'obj/{t}/obj_score'].view(-1).tolist()}")
for k in ("loss_mask", "loss_dice", "loss_iou", "total_loss"):
    print(k, float(losses[k]), float(g[f"loss/{k}"]))
grads = grads_by_name(model)
rows = []
for k in g:
    if k.startswith("gnorm/"):
        n = k[6:]
        ref = float(g[k])
        got = float(grads[n].double().norm()) if n in grads else float("nan")
        rows.append((abs(got - ref) / (ref + 1e-12), n, got, ref))
rows.sort(reverse=True)
print("worst gradient norms (rel err, name, got, ref):")
for r in rows[:25]:
    print(f"  {r[0]:.3e} {r[1]} {r[2]:.6e} {r[3]:.6e}")
print("params with grads:", len(rows), "median rel err", sorted(x[0] for x in rows)[len(rows) // 2])
