"""Write profiles/<round>_flash_fwd_pmc.json from the FETCH_SIZE / WRITE_SIZE passes of
tools/gpu_prof.sh TAG (gpurun_out/TAG_fetch, gpurun_out/TAG_write).
  python tools/pmc_json.py TAG profiles/r01_flash_fwd_pmc.json"""
import collections
import csv
import glob
import json
import sys


def collect(pattern, counter):
    by = collections.defaultdict(list)
    for f in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                by[r.get("Grid_Size", r.get("Grid_Size_X", "?"))].append(float(r["Counter_Value"]))
    vals = [v for vs in by.values() for v in vs]
    return {"launches": len(vals), "avg_kb": sum(vals) / max(len(vals), 1),
            "by_grid": {g: sum(v) / len(v) for g, v in sorted(by.items())}}


def main(tag, out):
    fetch = collect(f"gpurun_out/{tag}_fetch/**/*counter_collection.csv", "FETCH_SIZE")
    write = collect(f"gpurun_out/{tag}_write/**/*counter_collection.csv", "WRITE_SIZE")
    doc = {"FETCH_SIZE": fetch, "WRITE_SIZE": write, "kernel": "flash_fwd_kernel<256>",
           "command": "rocprofv3 --pmc FETCH_SIZE (resp. WRITE_SIZE) --kernel-include-regex flash_fwd_kernel -- "
                      f"python3 bench.py --steps 1 --warmup 1 --cpu-baseline 0 --no-prof (tools/gpu_prof.sh {tag})",
           "correction": "hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: gfx950 FETCH_SIZE reports half the bytes "
                         "of 16-B/lane streaming reads (MI355X_MICROARCH.md, HBM section); Infinity-Cache hits are "
                         "counted",
           "bytes_per_launch": (2 * fetch["avg_kb"] + write["avg_kb"]) * 1024}
    json.dump(doc, open(out, "w"), indent=1)
    print(json.dumps({k: doc[k] for k in ("bytes_per_launch",)}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
