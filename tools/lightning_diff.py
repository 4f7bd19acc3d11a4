"""Which parameters' gradients differ between StepRunner runs and the Lightning graph path after each
accumulation window at the bench workload -- the diagnosis behind tests/test_lightning_gpu.py.
    python tools/lightning_diff.py [ACC] [RUNS]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "sam2-video-training_amd"))

import torch  # noqa: E402

import test_lightning_gpu as T  # noqa: E402
from test_configs_gpu import _clips, _module  # noqa: E402


def names(m):
    arena = m.model.arena
    out = []
    for n, p in m.model.named_parameters():
        g = getattr(p, "_s2h_grad", None)
        if g is not None:
            out.append((n, (g.data_ptr() - arena.grad.data_ptr()) // g.element_size(), g.numel()))
    return out


def report(tag, a, b, nm):
    d = [(n, float((a[o:o + k] - b[o:o + k]).abs().max())) for n, o, k in nm
         if not torch.equal(a[o:o + k], b[o:o + k])]
    print(f"{tag}: {len(d)} of {len(nm)} parameters differ; first (in arena order): {d[:4]}", flush=True)
    if d and os.environ.get("LD_SAME"):
        bad = {n for n, _ in d}
        print("   equal:", [n for n, _, _ in nm if n not in bad], flush=True)


def runner(clips, acc):
    from sam2_video.training.trainer import StepRunner
    m = _module("base_plus", 512, lr=1e-4, clip=1.0)
    run = StepRunner(m, total_steps=2, graph=True, accumulate_grad_batches=acc, gradient_clip_val=1.0)
    grads, caps = [], []
    for i, c in enumerate(clips):
        n = len(run._graphs)
        run(c)
        if len(run._graphs) != n:
            caps.append(i)
        if (i + 1) % acc == 0:
            grads.append(m.model.arena.grad_region().clone())
    torch.cuda.synchronize()
    print(f"runner: captures at micro-steps {caps}", flush=True)
    return grads


def main():
    acc = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    runs = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    T.ACC = acc
    clips = _clips(range(300, 300 + acc), 8, 512, 13, 13)
    nm = names(_module("base_plus", 512))
    gs = [runner(clips + clips, acc) for _ in range(runs)]
    gl, _, _ = T._lightning_windows(clips + clips)
    for w in range(2):
        for r in range(1, runs):
            report(f"window {w} runner 0 vs runner {r}", gs[0][w], gs[r][w], nm)
        report(f"window {w} runner {runs - 1} vs lightning", gs[-1][w], gl[w], nm)


if __name__ == "__main__":
    main()
