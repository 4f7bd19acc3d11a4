"""Per-kernel GPU time of one replayed step in two rocprofv3 --kernel-trace databases (A, B): the
kernels whose total time changed most between two library builds.
    python tools/trace_diff.py A.db B.db [--top 30]"""
import argparse
import collections
import re
import sqlite3


def step_kernels(db, marker="adamw_kernel", back=2):
    rows = sqlite3.connect(db).execute("select name, start, end from kernels order by start").fetchall()
    ends = [i for i, r in enumerate(rows) if marker in r[0]]
    i0, i1 = ends[-back - 1] + 1, ends[-back] + 1
    agg, cnt = collections.Counter(), collections.Counter()
    for n, s, e in rows[i0:i1]:
        k = re.sub(r"\(.*", "", n)
        agg[k] += e - s
        cnt[k] += 1
    return agg, cnt, rows[i1 - 1][2] - rows[i0][1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("a")
    ap.add_argument("b")
    ap.add_argument("--top", type=int, default=30)
    x = ap.parse_args()
    (ka, ca, sa), (kb, cb, sb) = step_kernels(x.a), step_kernels(x.b)
    print(f"step span A {sa / 1e6:.3f} ms  B {sb / 1e6:.3f} ms;  kernel time A {sum(ka.values()) / 1e6:.3f}  "
          f"B {sum(kb.values()) / 1e6:.3f} ms")
    names = set(ka) | set(kb)
    d = sorted(names, key=lambda n: -abs(kb[n] - ka[n]))
    for n in d[:x.top]:
        print(f"{(kb[n] - ka[n]) / 1e3:+9.1f} us  A {ka[n] / 1e3:9.1f} ({ca[n]:4d})  B {kb[n] / 1e3:9.1f} ({cb[n]:4d})  {n[:110]}")


if __name__ == "__main__":
    main()
