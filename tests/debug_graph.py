"""Debug helper (not a test): per-parameter gradient differences, eager vs graphed step."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "sam2-video-training_amd"))
import torch  # noqa: E402

from test_graph_gpu import _clips, _runner  # noqa: E402


def grads(graph, clip, steps=1):
    module, run = _runner(graph, 0.0, lr=0.0)
    for _ in range(steps):
        run(clip)
    torch.cuda.synchronize()
    out = {}
    for n, p in module.model.named_parameters():
        g = getattr(p, "_s2h_grad", None)
        if g is not None:
            out[n] = g.detach().float().cpu().clone()
    return out


clip = _clips([11])[0]
e1, e2, g1 = grads(False, clip), grads(False, clip), grads(True, clip)
g2 = grads(True, clip, steps=2)
rows = []
for n in e1:
    d_ee = (e1[n] - e2[n]).abs().max().item()
    d_eg = (e1[n] - g1[n]).abs().max().item()
    d_gg = (g1[n] - g2[n]).abs().max().item()
    rows.append((d_eg, d_ee, d_gg, e1[n].abs().max().item(), n))
rows.sort(reverse=True)
for r in rows[:25]:
    print("eg %.3e ee %.3e gg %.3e max %.3e %s" % r)
