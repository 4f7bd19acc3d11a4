"""Counter passes of tools/gpu_prof2.sh -> profiles/<round>_{gemm,attn_bwd,attn_fwd}_pmc.json.

Per kernel name and grid (so self- and cross-attention launches are separate rows): dispatches per
step, FETCH_SIZE / WRITE_SIZE (KiB per dispatch), HBM bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024
(gfx950 FETCH_SIZE counts half the bytes of 16-B/lane streaming reads, MI355X_MICROARCH.md HBM
section; Infinity-Cache hits included) and the SQ counters.  Per family, `bytes_per_launch` = HBM
bytes of one training step / the family's host-level launches per step (the bench's roofline unit:
one launch = one ABI call, e.g. di + dQ + dK/dV kernels of one attention backward; the launch counts
come from the bench line of the same call).
  python tools/pmc_family.py TAG STEPS BENCH_LOG OUT_PREFIX"""
import collections
import csv
import glob
import json
import re
import sys

FAMILIES = {"gemm": ("GEMM", r"gemm"), "attn_bwd": ("attention backward", r"flash_bwd|attn_bwd"),
            "attn_fwd": ("attention forward", r"flash_fwd|flash_combine|attn_fwd")}


def main(tag, steps, bench_log, prefix):
    steps = int(steps)
    line = [ln for ln in open(bench_log) if ln.startswith("{")][-1]
    rl = json.loads(line)["roofline"]
    fams = rl["families"]
    # host-level launches (one ABI call = one launch: the unit of the bench line's alg_bytes_per_launch);
    # the trace-based families count kernels, the event-based ones count launches
    ev = rl.get("event_based", {}).get("families", {})
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"gpurun_out/{tag}_pmc*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            key = (r["Kernel_Name"].split("(")[0].replace("void ", ""), int(r["Grid_Size"]), int(r["Workgroup_Size"]))
            per[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for short, (name, rx) in FAMILIES.items():
        rows, fetch, write = [], 0.0, 0.0
        for (kn, grid, wg), cs in per.items():
            if not re.search(rx, kn):
                continue
            n = max(len(v) for v in cs.values())
            row = {"kernel": kn, "grid": grid, "workgroup": wg, "dispatches_per_step": n / steps}
            row.update({c: sum(v) / len(v) for c, v in cs.items()})
            if "FETCH_SIZE" in row and "WRITE_SIZE" in row:
                row["hbm_bytes_per_dispatch"] = (2 * row["FETCH_SIZE"] + row["WRITE_SIZE"]) * 1024
            if "SQ_BUSY_CYCLES" in row and "SQ_VALU_MFMA_BUSY_CYCLES" in row and "GRBM_GUI_ACTIVE" in row:
                row["mfma_busy_frac"] = row["SQ_VALU_MFMA_BUSY_CYCLES"] / max(row["GRBM_GUI_ACTIVE"] / 8 * 256 * 4, 1)
            fetch += sum(cs.get("FETCH_SIZE", []))
            write += sum(cs.get("WRITE_SIZE", []))
            rows.append(row)
        if not rows:
            continue
        rows.sort(key=lambda r: -r.get("hbm_bytes_per_dispatch", 0) * r["dispatches_per_step"])
        step_bytes = (2 * fetch + write) * 1024 / steps
        launches = ev.get(name, {}).get("launches_per_step") or fams.get(name, {}).get("launches_per_step", 0)
        doc = {"family": name, "tag": tag, "steps": steps, "launches_per_step": launches,
               "hbm_bytes_per_step": step_bytes, "bytes_per_launch": step_bytes / max(launches, 1),
               "correction": "hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE = half the bytes of "
                             "16-B/lane streaming reads; MI355X_MICROARCH.md HBM section); mfma_busy_frac = "
                             "SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 256 CUs * 4 SIMDs)",
               "command": f"bash tools/gpu_prof2.sh {tag}: rocprofv3 --pmc <one set per pass> --kernel-include-regex "
                          f"'gemm|flash|attn_' -- python3 tools/step_once.py {steps}",
               "kernels": rows}
        out = f"{prefix}_{short}_pmc.json"
        json.dump(doc, open(out, "w"), indent=1)
        print(out, f"{step_bytes / 1e9:.3f} GB/step", f"{doc['bytes_per_launch'] / 1e6:.2f} MB/launch")


if __name__ == "__main__":
    main(*sys.argv[1:5])
