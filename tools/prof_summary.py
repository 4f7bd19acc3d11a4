"""Summarise a rocprofv3 `--kernel-trace --stats` output directory into a per-kernel table.

Reads either the rocpd SQLite database (`*_results.db`, rocprofv3's default output) or the
CSV `*_kernel_stats.csv` (`--output-format csv`), and writes a CSV with
name, calls, total_ms, avg_us, pct, sorted by total time.

  python tools/prof_summary.py gpurun_out/prof2 profiles/r01_bench_kernel_stats.csv [--top 40]
"""
import argparse
import csv
import glob
import os
import sqlite3
import sys


def load(path):
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("dst")
    ap.add_argument("--top", type=int, default=0)
    a = ap.parse_args()
    rows = sorted(load(a.src), key=lambda r: -r[2])
    total = sum(r[2] for r in rows)
    if a.top:
        rows = rows[: a.top]
    os.makedirs(os.path.dirname(os.path.abspath(a.dst)), exist_ok=True)
    with open(a.dst, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["name", "calls", "total_ms", "avg_us", "pct"])
        for n, c, t in rows:
            w.writerow([n, c, f"{t:.3f}", f"{1e3 * t / c:.2f}", f"{100 * t / total:.2f}"])
    print(f"total kernel time {total:.1f} ms")
    for n, c, t in rows[:25]:
        print(f"{t:9.2f} ms {100 * t / total:5.1f}% {c:6d} {1e3 * t / c:9.1f} us  {n[:110]}")


if __name__ == "__main__":
    main()
