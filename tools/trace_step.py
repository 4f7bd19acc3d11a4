"""Summarise one training step of a rocprofv3 --kernel-trace csv: the step between the last two
AdamW launches, kernel time by name and by (name, grid), busy vs span."""
import collections
import csv
import sys


def main(path, top=40):
    tr = list(csv.DictReader(open(path)))
    tr.sort(key=lambda r: int(r["Start_Timestamp"]))
    ad = [i for i, r in enumerate(tr) if "adamw" in r["Kernel_Name"]]
    seg = tr[ad[-2] + 1:ad[-1] + 1]
    t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
    busy, cs, ce = 0, None, None
    for r in seg:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if ce is None or s > ce:
            if ce is not None:
                busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    print(f"step: {len(seg)} kernels, span {(t1 - t0) / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms")
    by = collections.defaultdict(lambda: [0, 0])
    byg = collections.defaultdict(lambda: [0, 0])
    for r in seg:
        k = r["Kernel_Name"].split("(")[0][:60]
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        by[k][0] += 1
        by[k][1] += d
        g = (k, r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
        byg[g][0] += 1
        byg[g][1] += d
    print("--- by kernel")
    for k, v in sorted(by.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{v[1] / 1e6:8.2f} ms {v[0]:5d} {v[1] / v[0] / 1e3:8.1f} us  {k}")
    print("--- by kernel and grid")
    for k, v in sorted(byg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{v[1] / 1e6:8.2f} ms {v[0]:5d} {v[1] / v[0] / 1e3:8.1f} us  {k[0][:45]} grid {k[1]}x{k[2]}x{k[3]}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40)
