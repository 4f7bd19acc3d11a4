"""Weight-gradient GEMM (dW[N, K] += dY[rows, N]^T X[rows, K] into the fp32 gradient arena) per-launch
time on the step's shapes (graph replays, tools/gemm_graph_bench.py): the deterministic kernel
(csrc/gemm_wgrad.hip, round 5) against the split-K fp32-atomic tilings it replaced.  Also checks it
against the fp32 product and bit-for-bit across repeats.   GPU only.   python tools/wgrad_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402
from gemm_graph_bench import graph_time  # noqa: E402

from sam2_video.kernels import _lib, ops  # noqa: E402

# (N out, K in, rows) -- the step's long-reduction weight gradients (profiles/r04_v27_kernel_table.txt)
SHAPES = [(256, 2048, 93184), (2048, 256, 93184), (256, 256, 93184), (768, 256, 93184), (256, 72, 93184),
          (256, 64, 374192), (128, 256, 106496), (1792, 448, 8192), (448, 1792, 8192), (1344, 448, 14112),
          (448, 448, 14112), (896, 224, 32768), (224, 896, 32768), (112, 448, 131072), (448, 112, 131072),
          (2688, 896, 3528), (896, 896, 3528), (32, 256, 131072)]
CFGS = ((7, "128x64-atomic"), (-2, "auto-atomic"), (0, "det"))


def main():
    bf = torch.bfloat16
    ws = ops.wgrad_workspace("cuda")
    h = _lib.lib()
    for N, K, R in SHAPES:
        torch.manual_seed(0)
        dy = torch.randn(R, N, device="cuda", dtype=bf)
        x = torch.randn(R, K, device="cuda", dtype=bf)
        dw = torch.zeros(N, K, device="cuda")
        db = torch.zeros(N, device="cuda")
        row = f"wgrad {N}x{K} over {R} |"
        flops = 2.0 * N * K * R
        for c, nm in CFGS:
            h.s2h_wgrad_workspace(ws.data_ptr(), ops.WGRAD_WS_BYTES, 0 if c == -2 else 1024)
            h.s2h_gemm_config(max(c, 0))
            t = graph_time(lambda: ops.linear_wgrad(dy, x, dw, db=db))
            row += f" {nm} {t:6.1f} us ({flops / t / 1e6:5.0f} TF/s)"
        h.s2h_gemm_config(0)
        h.s2h_wgrad_workspace(ws.data_ptr(), ops.WGRAD_WS_BYTES, 1024)
        ref = dy.float().t() @ x.float()
        outs = []
        for r in range(3):
            dw.fill_(0.5)
            db.fill_(0.25)
            ops.linear_wgrad(dy, x, dw, db=db)
            torch.cuda.synchronize()
            outs.append((dw.clone(), db.clone()))
        err = ((outs[0][0] - 0.5 - ref).abs().max() / ref.abs().max()).item()
        berr = ((outs[0][1] - 0.25 - dy.float().sum(0)).abs().max() / dy.float().sum(0).abs().max()).item()
        same = all(torch.equal(outs[0][0], o[0]) and torch.equal(outs[0][1], o[1]) for o in outs[1:])
        print(row + f" | rel err {err:.1e} bias {berr:.1e} repeat-identical {same}", flush=True)


if __name__ == "__main__":
    main()
