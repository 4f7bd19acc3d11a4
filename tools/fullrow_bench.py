"""Full-row GEMM tilings (round 4: CFG 25-28, a workgroup owns 64 rows x the whole N <= 256 output)
against the automatic choice on the step's N <= 256 shapes: graph-replayed time per launch, hot and
cold caches, each epilogue the step uses; results must be bit-identical to the automatic tiling.
    python tools/fullrow_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

from gemm_graph_bench import graph_time, graph_time_cold  # noqa: E402
from sam2_video.kernels import _lib, ops  # noqa: E402

SHAPES = [(13312, 256, 256), (13312, 128, 256), (13312, 256, 72), (13312, 256, 2048), (13312, 256, 1024),
          (93184, 256, 256), (13312, 256, 128), (53248, 128, 256), (104, 256, 256)]
CFGS = [0, 25, 26, 27, 28]


def main():
    bf = torch.bfloat16
    torch.manual_seed(0)
    L = _lib.lib()
    ops.rng_offset("cuda").fill_(1)
    for M, N, K in SHAPES:
        x = torch.randn(M, K, device="cuda", dtype=bf)
        w = torch.randn(N, K, device="cuda", dtype=bf) * 0.05
        b = torch.randn(N, device="cuda")
        r = torch.randn(M, N, device="cuda", dtype=bf)
        out = torch.empty(M, N, device="cuda", dtype=bf)
        epis = {"bias": lambda: ops.linear(x, w, b, out=out),
                "res+drop": lambda: ops.linear(x, w, b, out=out, residual=r, drop_p=0.1, seed=3)}
        for en, fn in epis.items():
            row = f"{M}x{N}x{K:<5} {en:9s}"
            ref = None
            for c in CFGS:
                if c in (25, 27, 28) and N != 256 or c == 26 and N != 128:
                    continue
                L.s2h_gemm_config(c)
                out.fill_(float("nan"))
                fn()
                torch.cuda.synchronize()
                if ref is None:
                    ref = out.clone()
                same = "" if torch.equal(out, ref) else "(DIFF)"
                row += f" c{c}:{graph_time(fn):6.1f}/{graph_time_cold(fn):6.1f}{same}"
            L.s2h_gemm_config(0)
            print(row, flush=True)
        if N in (128, 256) and M >= 1000:
            # the model's pair: y = linear(o) with dropout, then LN(x + y) and x + y in one LN launch,
            # against the fused full-row launch
            g, be = torch.rand(N, device="cuda") + 0.5, torch.randn(N, device="cuda") * 0.1
            y = torch.empty(M, N, device="cuda", dtype=bf)
            xs = torch.empty(M, N, device="cuda", dtype=bf)
            mean = torch.empty(M, device="cuda")
            rstd = torch.empty(M, device="cuda")

            def unfused():
                o = ops.linear(x, w, b, out=out, drop_p=0.1, seed=3)
                ops.layernorm_fwd(r, g, be, 1e-5, y=y, add=o, xsum=xs)

            def fused():
                ops.linear_add_ln(x, w, b, r, g, be, 1e-5, drop_p=0.1, seed=3, xsum=xs, y=y, mean=mean, rstd=rstd)
            print(f"{M}x{N}x{K:<5} linear+add+LN   unfused {graph_time(unfused):6.1f}/{graph_time_cold(unfused):6.1f}"
                  f"  fused {graph_time(fused):6.1f}/{graph_time_cold(fused):6.1f}", flush=True)


if __name__ == "__main__":
    main()
