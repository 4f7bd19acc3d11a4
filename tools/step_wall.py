"""Where the graphed bench step's wall time goes: host issue time of one step (runner call until
it returns), GPU time between events at the step's ends, wall time per step of K back-to-back
steps, and each captured graph replayed alone (phase-1 graph, each backbone segment graph).
Compare against the kernel-time sum of the rocprof stats: GPU time well above it is bubbles
between kernels inside the graphs; wall above GPU time is host-bound issue.
    python tools/step_wall.py [--steps 10]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    from sam2_video.data.synthetic import make_clip, sam2_collate_fn
    from sam2_video.model.sam2model import SAM2Model
    from sam2_video.training.trainer import SAM2LightningModule, StepRunner
    ALL = ["image_encoder", "memory_attention", "memory_encoder", "mask_decoder", "prompt_encoder"]
    model = SAM2Model(None, "base_plus@512", trainable_modules=ALL, compute_dtype="bf16")
    loss_cfg = {"weight_dict": {"loss_mask": 20, "loss_dice": 1, "loss_iou": 1, "loss_class": 0},
                "supervise_all_iou": True, "iou_use_l1_loss": True}
    module = SAM2LightningModule(model, loss_cfg, {"type": "AdamW", "lr": 4e-6}, {"enabled": False})
    module.setup("fit", "cuda")
    run = StepRunner(module, 100, graph=True)
    batches = [sam2_collate_fn([make_clip(i, 8, 512, 13, 13)]).to("cuda") for i in range(2)]
    for i in range(3):
        run(batches[i % 2])
    torch.cuda.synchronize()
    issue, gpu = [], []
    t0 = time.perf_counter()
    for i in range(a.steps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        h0 = time.perf_counter()
        e0.record()
        run(batches[i % 2])
        e1.record()
        issue.append(time.perf_counter() - h0)
        gpu.append((e0, e1))
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.steps
    g = sum(e0.elapsed_time(e1) for e0, e1 in gpu) / a.steps
    print(f"wall/step {wall * 1e3:8.2f} ms   gpu/step {g:8.2f} ms   host issue/step "
          f"{1e3 * sum(issue) / len(issue):8.2f} ms (max {1e3 * max(issue):.2f})", flush=True)
    ent = next(iter(run._graphs.values()))

    def alone(fn, n=5):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        h0 = time.perf_counter()
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        h = (time.perf_counter() - h0) / n
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n, h * 1e3

    t, h = alone(ent["graph"].replay)
    print(f"phase-1 graph alone   gpu {t:8.2f} ms   host launch {h:6.2f} ms", flush=True)
    for k, (rep, rank, _) in enumerate(ent["segs"]):
        t, h = alone(rep)
        print(f"segment {k} (rank {rank}) gpu {t:8.2f} ms   host launch {h:6.2f} ms", flush=True)
    t, h = alone(lambda: module.optimizer.step(lr=1e-9))
    print(f"optimizer             gpu {t:8.2f} ms   host {h:6.2f} ms", flush=True)
    t, h = alone(lambda: model.host_prompt_plan(batches[0]))
    print(f"host prompt plan                        host {h:6.2f} ms", flush=True)


if __name__ == "__main__":
    main()
