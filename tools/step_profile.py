"""Per-step kernel table of the timed graph replays from a rocprofv3 `--kernel-trace --stats -f csv`
run of bench.py: only the dispatches between the two trace markers bench.py launches around its
timed steps (s2h_trace_marker_kernel) count -- no setup copies, no warm-up, no profiled eager step.
`dir` may also be the per-kernel CSV bench.py itself writes from its traced run (--trace-out), so the
table and the bench line come from one trace.

Writes a CSV (name, calls, calls_per_step, total_ms, ms_per_step, avg_us, pct) and prints the
per-family split; with --bench <bench JSON line> it also recomputes the roofline's dominant-kernel
fraction from the trace alone: alg_flop_per_launch (bench line) / avg duration (trace) / peak.

  python tools/step_profile.py gpurun_out/r04_kt profiles/r04_v2_kernel_stats.csv --steps 10 \
      --bench gpurun_out/r04_kt_bench.log
"""
import argparse
import csv
import glob
import json
import os
import re
import sqlite3
import sys

FAMILIES = [("GEMM (bf16)", r"gemm16[ag]?_kernel|gemm_kernel<|gemm_wg|gemm_split|ffn_"), ("GEMM (MX-fp8)", r"gemm_mx8|mx8_quant"),
            ("flash forward", r"flash_fwd|flash_combine"), ("flash backward", r"flash_bwd"),
            ("window / decoder attention", r"attn_"), ("LayerNorm", r"ln_|layernorm"),
            ("loss / merge / eval", r"mask_|bce_|group_"), ("optimizer", r"adamw|sumsq|norm_finalize"),
            ("stock torch", r"at::|elementwise_kernel|vectorized|__amd_rocclr|Memset|fill")]


def load_region(path, verbose=True):
    """per-kernel (name, calls, total ms) of the dispatches between bench.py's two trace markers
    (s2h_trace_marker_kernel) in a rocprofv3 kernel-trace CSV; None if there is no such trace"""
    traces = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
    if not traces:
        return None
    rows = []
    with open(traces[0]) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if "s2h_trace_marker_kernel" in r[2]]
    if len(marks) < 2:
        raise ValueError(f"{traces[0]}: {len(marks)} trace markers (bench.py launches one before and one after the "
                         "timed steps)")
    agg = {}
    for st, en, name in rows[marks[0] + 1:marks[1]]:
        a = agg.setdefault(name, [0, 0.0])
        a[0] += 1
        a[1] += (en - st) / 1e6
    span = (rows[marks[1]][0] - rows[marks[0]][1]) / 1e6
    if verbose:
        print(f"timed region: {marks[1] - marks[0] - 1} dispatches, {span:.2f} ms wall between the markers")
    return [(n, c, t) for n, (c, t) in agg.items()]


def load(path):
    if os.path.isfile(path):  # a per-kernel CSV written by write_stats (bench.py --trace-out): totals
        out = []
        with open(path) as f:
            next(f)
            for r in csv.DictReader(f):
                out.append((r["name"], int(r["calls"]), float(r["total_ms"])))
        return out
    reg = load_region(path)
    if reg is not None:
        return reg
    dbs = glob.glob(os.path.join(path, "**", "*_results.db"), recursive=True)
    if dbs:
        con = sqlite3.connect(dbs[0])
        rows = con.execute("select name, count(*), sum(duration) from kernels group by name").fetchall()
        return [(n, int(c), float(t) / 1e6) for n, c, t in rows]
    stats = glob.glob(os.path.join(path, "**", "*kernel_stats.csv"), recursive=True)
    if not stats:
        sys.exit(f"no rocprofv3 output under {path}")
    out = []
    with open(stats[0]) as f:
        for r in csv.DictReader(f):
            out.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e6))
    return out


def short(name):
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\((GemmArgs16|GemmArgs16Ln|FlashArgs|FlashBwdArgs|Mx8Args|Mx8QArgs)\)$", "", name)
    # gemm16g_kernel's argument-block parameter (GemmArgs16 / GemmArgs16Ln, gemm_bf16.h): bench.py's
    # kernel_name() spells the tiling without it
    return re.sub(r", GemmArgs16(Ln)?>$", ">", name)


def family_of(name):
    return next((fn for fn, pat in FAMILIES if re.search(pat, name)), "element-wise / other")


def write_stats(rows, steps, out):
    """the per-kernel CSV of `rows` [(name, calls, total ms)] over `steps` timed steps"""
    rows = sorted(rows, key=lambda r: -r[2])
    tot = sum(r[2] for r in rows)
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow([f"# rocprofv3 kernel trace of {steps} timed graph-replayed steps (the dispatches between "
                    f"bench.py's trace markers); {tot / steps:.3f} ms of kernel time per step"])
        w.writerow(["name", "calls", "calls_per_step", "total_ms", "ms_per_step", "avg_us", "pct"])
        for n, c, t in rows:
            w.writerow([short(n), c, round(c / steps, 2), round(t, 4), round(t / steps, 4),
                        round(1e3 * t / c, 3), round(100 * t / tot, 2)])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("out")
    ap.add_argument("--steps", type=int, required=True, help="timed steps between the trace markers")
    ap.add_argument("--bench", default=None)
    ap.add_argument("--peak", type=float, default=2500.0)
    a = ap.parse_args()
    rows = sorted(load(a.dir), key=lambda r: -r[2])
    tot = sum(r[2] for r in rows)
    write_stats(rows, a.steps, a.out)
    fam = {}
    for n, c, t in rows:
        k = family_of(n)
        fam[k] = fam.get(k, 0.0) + t
    print(f"{tot / a.steps:.3f} ms kernel time per step over {a.steps} steps, {sum(r[1] for r in rows) / a.steps:.0f} "
          "kernels per step")
    for k, t in sorted(fam.items(), key=lambda kv: -kv[1]):
        print(f"  {k:28s} {t / a.steps:8.3f} ms/step  {100 * t / tot:5.1f} %")
    if a.bench:
        line = [x for x in open(a.bench).read().splitlines() if x.startswith("{")][-1]
        dk = json.loads(line)["roofline"]["dominant_kernel"]
        hit = [r for r in rows if short(r[0]) == dk["name"]]
        if hit:
            n, c, t = hit[0]
            avg = 1e3 * t / c
            frac = dk["alg_flop_per_launch"] / (avg * 1e-6) / 1e12 / a.peak
            print(f"dominant kernel {dk['name']}: trace {c / a.steps:.1f} calls/step avg {avg:.2f} us "
                  f"(bench events {dk['avg_us']} us, {dk['launches_per_step']} calls); "
                  f"{dk['alg_flop_per_launch']:.4g} flop/launch -> frac {frac:.4f} (bench {dk['frac']})")
        else:
            print(f"dominant kernel {dk['name']} not in the trace")


if __name__ == "__main__":
    main()
