"""Digest of one bf16 B+ 256^2 training step on the reference's fixture clip (tests/golden): the loss,
every stage's mask logits and every parameter gradient, hashed bit for bit.  Run once per build
(S2H_LIB_PATH selects an older one) and compare the lines: a kernel change that claims the same sums in
the same order must print the same digest.
    python tools/arena_digest.py [GOLDEN]"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))

import torch  # noqa: E402


def main():
    from step_harness import build_model, golden_batch, grads_by_name, load_golden, run_step
    name = sys.argv[1] if len(sys.argv) > 1 else "bplus256_point_all"
    batch = golden_batch(load_golden(name)).to("cuda")
    model = build_model("base_plus", 256, ["image_encoder", "memory_attention", "memory_encoder", "mask_decoder",
                                           "prompt_encoder"], "point", dtype="bf16")
    stages, _, losses, _ = run_step(model, batch)
    torch.cuda.synchronize()
    h = hashlib.sha256()
    h.update(torch.tensor(float(losses["total_loss"])).numpy().tobytes())
    for s in stages:
        h.update(s["pred_masks"].detach().float().cpu().numpy().tobytes())
    grads = grads_by_name(model)
    for n in sorted(grads):
        h.update(n.encode())
        h.update(grads[n].detach().float().cpu().numpy().tobytes())
    lib = os.path.basename(os.path.dirname(os.environ.get("S2H_LIB_PATH", "default/x")))
    print(f"digest {lib} {name} loss {float(losses['total_loss']):.9g} grads {len(grads)} {h.hexdigest()}")


if __name__ == "__main__":
    main()
