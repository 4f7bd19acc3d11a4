"""Memory-attention FFN backward (input-gradient side) and forward: the one-launch kernels (csrc/ffn.hip)
against the two GEMMs each replaces (dH with the ReLU/dropout mask in the epilogue, then dX = dH W1), graph-replayed
at the frame-batched bench shape.   GPU only.   python tools/ffn_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402
from gemm_graph_bench import graph_time  # noqa: E402

from sam2_video.kernels import ops  # noqa: E402


def main():
    bf = torch.bfloat16
    for R, H in ((93184, 2048), (13312, 2048)):
        torch.manual_seed(0)
        dy = torch.randn(R, 256, device="cuda", dtype=bf)
        w2 = (torch.randn(256, H, device="cuda") / 45).to(bf)
        w1 = (torch.randn(H, 256, device="cuda") / 16).to(bf)
        hid = torch.relu(torch.randn(R, H, device="cuda")).to(bf)
        dh = torch.empty(R, H, device="cuda", dtype=bf)
        dx = torch.empty(R, 256, device="cuda", dtype=bf)
        alpha = 1 / 0.9
        t_f = graph_time(lambda: ops.ffn_bwd_dgrad(dy, w2, w1, hid, alpha, dh=dh, dx=dx))
        t_a = graph_time(lambda: ops.linear_dgrad(dy, w2, dx=dh, pre=hid, act="relu", alpha=alpha))
        t_b = graph_time(lambda: ops.linear_dgrad(dh, w1, dx=dx))
        flops = 2 * 2 * R * H * 256
        byts = 2 * (R * 256 + R * H + R * H + R * 256)
        print(f"ffn bwd R={R} H={H}: fused {t_f:7.1f} us ({flops / t_f / 1e6:5.0f} TF/s, {byts / t_f / 1e3:5.0f} GB/s)"
              f" | two GEMMs {t_a:7.1f} + {t_b:7.1f} = {t_a + t_b:7.1f} us", flush=True)
        x = torch.randn(R, 256, device="cuda", dtype=bf)
        b1 = torch.randn(H, device="cuda") * 0.1
        b2 = torch.randn(256, device="cuda") * 0.1
        w1f = (torch.randn(H, 256, device="cuda") / 16).to(bf)
        w2f = (torch.randn(256, H, device="cuda") / 45).to(bf)
        y = torch.empty(R, 256, device="cuda", dtype=bf)
        f_f = graph_time(lambda: ops.ffn_fwd(x, w1f, b1, w2f, b2, 0.1, 11, 0, 12, 0, hid=dh, y=y))
        f_a = graph_time(lambda: ops.linear(x, w1f, b1, act="relu", drop_p=0.1, seed=11, out=dh))
        f_b = graph_time(lambda: ops.linear(dh, w2f, b2, drop_p=0.1, seed=12, out=y))
        print(f"ffn fwd R={R} H={H}: fused {f_f:7.1f} us ({flops / f_f / 1e6:5.0f} TF/s) | two GEMMs {f_a:7.1f} + "
              f"{f_b:7.1f} = {f_a + f_b:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
