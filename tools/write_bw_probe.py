"""Write bandwidth the step's GEMM epilogues can expect: cold-cache (graph_time_cold: after a 512 MB
dirty scrub) and hot graph time of plain fills / copies of the 13312x2048 / 93184x256 bf16 outputs.
    python tools/write_bw_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

from gemm_graph_bench import graph_time, graph_time_cold  # noqa: E402


def main():
    for M, N in ((13312, 2048), (93184, 256), (13312, 256)):
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        src = torch.randn(M, N, device="cuda").to(torch.bfloat16)
        mb = out.numel() * 2 / 1e6
        row = f"{M}x{N} ({mb:.1f} MB)"
        for nm, fn in (("fill", lambda: out.fill_(1.0)), ("copy", lambda: out.copy_(src)),
                       ("read", lambda: src.sum(dtype=torch.float32))):
            tc, th = graph_time_cold(fn), graph_time(fn)
            row += f"  {nm}: cold {tc:6.1f} us ({mb / tc:5.2f} TB/s) hot {th:6.1f} us"
        print(row, flush=True)


if __name__ == "__main__":
    main()
