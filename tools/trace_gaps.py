"""Idle time between kernels of the timed graph replays, from a rocprofv3 --kernel-trace database
(rocpd SQLite, ROCm 7): per replayed step, the kernels' busy time (union of [start, end)) and the
gaps between one kernel's end and the next one's start.  A gap is dispatch / dependency latency the
GPU spends with no kernel of the step running.
    python tools/trace_gaps.py <results.db> [--steps N]"""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=3, help="replayed steps at the end of the trace to analyse")
    ap.add_argument("--marker", default="adamw_kernel", help="kernel that ends a step")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    ends = [i for i, r in enumerate(rows) if a.marker in r[0]]
    if len(ends) < a.steps + 1:
        raise SystemExit(f"only {len(ends)} '{a.marker}' dispatches in the trace")
    for s in range(a.steps):
        i0, i1 = ends[-a.steps - 1 + s] + 1, ends[-a.steps + s] + 1
        ks = rows[i0:i1]
        t0, t1 = ks[0][1], ks[-1][2]
        busy, cur_s, cur_e = 0, ks[0][1], ks[0][2]
        gaps = collections.Counter()
        gap_n = 0
        for name, st, en in ks[1:]:
            if st > cur_e:
                busy += cur_e - cur_s
                g = st - cur_e
                gaps["< 2 us" if g < 2000 else "2-5 us" if g < 5000 else "5-20 us" if g < 20000 else ">= 20 us"] += g
                gap_n += 1
                cur_s, cur_e = st, en
            else:
                cur_e = max(cur_e, en)
        busy += cur_e - cur_s
        span = t1 - t0
        print(f"step {s}: {len(ks)} kernels, span {span / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms, "
              f"idle {(span - busy) / 1e6:.2f} ms in {gap_n} gaps "
              f"({', '.join(f'{k}: {v / 1e6:.2f} ms' for k, v in sorted(gaps.items()))})", flush=True)


if __name__ == "__main__":
    main()
