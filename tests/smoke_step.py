"""__graft_entry__.smoke(): one small training step (forward + loss + backward) of the HIP
path on cuda:0, checked against the CPU oracle on the same seeded clip and weights."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, os.path.join(ROOT, "sam2-video-training_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def run_smoke():
    import torch

    import sam2_oracle as O
    from step_harness import ALL, build_model, run_step
    from sam2_video.data.synthetic import make_clip, sam2_collate_fn
    from sam2_video.model.configs import model_config
    from sam2_video.utils.init import synth_tensor

    assert torch.cuda.is_available(), "smoke needs the GPU"
    size, S, T, n_cat, n_obj = "tiny", 128, 2, 4, 2
    clip = make_clip(3, T, S, n_cat, n_obj)
    model = build_model(size, S, ALL, "point", dtype="fp32")
    stages, merged, losses, _ = run_step(model, sam2_collate_fn([clip]).to("cuda"))
    cfg = model_config(size, S)
    P = O.make_params(O.param_shapes(cfg), O.trainable_prefixes(ALL), synth_tensor, seed=0)
    o_stages, o_merged, _ = O.OracleSAM2(cfg, P).forward(clip["images"], clip["masks"])
    o_losses = O.multistep_loss(o_merged, clip["masks"])
    worst = max((s["pred_masks"].detach().cpu() - o["pred_masks"].detach()).abs().max().item()
                for s, o in zip(stages, o_stages))
    dl = abs(float(losses["total_loss"].detach()) - float(o_losses["total_loss"].detach()))
    assert worst <= 1e-3, f"mask logits differ from the oracle by {worst}"
    assert dl <= 1e-4 * max(1.0, abs(float(o_losses["total_loss"].detach()))), f"loss differs by {dl}"
    print(f"smoke ok: max |logit diff| {worst:.2e}, |loss diff| {dl:.2e}")


if __name__ == "__main__":
    run_smoke()
