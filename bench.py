"""Headline benchmark: training clip-frames/s of the SAM2 video fine-tuning step
(BASELINE.json metric) on synthetic 512^2 8-frame clips, Hiera-B+, 13 objects,
bf16 compute, all five modules trainable (the north_star "Hiera fwd+bwd").

One step = SAM2LightningModule.training_step on one clip per rank (forward over
8 frames, category merge, focal/Dice/IoU loss) + backward + RCCL all-reduce of
the flat gradient arena (N > 1) + grad-norm clip + AdamW.  Inputs are resident
in HBM before the timed region.  Prints ONE JSON line on rank 0.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

The roofline (N = 1): before it touches the GPU, bench.py runs a copy of itself under
`rocprofv3 --kernel-trace` (--trace-child: same workload, --trace-steps timed replays between the
trace markers); per-family and dominant-kernel durations come from that trace of the timed replays,
algorithmic flops per launch from the in-library profiler's records of one eager step after the
timed region.  The event-bracketed durations of that eager step ride along under
roofline.event_based.  --trace-out writes the trace's per-kernel CSV (tools/step_profile.py reads it
with the same bench line).  --no-trace skips the traced run.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, chip-level parameters)
PEAK_FP8_TFLOPS = 5000.0  # dense block-scaled fp8 MFMA (same table; the MX-fp8 GEMM family is priced on it)
# algorithmic fwd+bwd TFLOP per clip-frame: config 2 all-trainable
# 13.75 TF / 8 frames, `mem` 11.14 TF / 8 frames
STEP_TF_PER_FRAME = {("base_plus", 512, 8, 13, "all"): 13.75 / 8, ("base_plus", 512, 8, 13, "mem"): 11.14 / 8}
ALL = ["image_encoder", "memory_attention", "memory_encoder", "mask_decoder", "prompt_encoder"]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--size", default="base_plus")
    ap.add_argument("--image-size", type=int, default=512)
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--objects", type=int, default=13)
    ap.add_argument("--dtype", default=None,
                    help="bf16 | fp32 | fp8 (MX-fp8 projections / FFN, kernels/fp8.py); default: bf16, "
                         "fp8 under --config 5 (--config 5 --dtype bf16 is its bf16 twin)")
    ap.add_argument("--config", type=int, default=2, choices=[2, 5],
                    help="BASELINE config preset: 2 = B+ 512^2 8 frames bf16 (the headline), "
                         "5 = B+ 512^2 16 frames MX-fp8 (long-memory stress)")
    ap.add_argument("--trainable", default="all", choices=["all", "mem"])
    ap.add_argument("--dropout", type=float, default=None, help="override dropout p (default: config, 0.1)")
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the CPU oracle on rank 0 at N=1")
    ap.add_argument("--cpu-frames", type=int, default=None,
                    help="frames of the CPU baseline sample clip (default: the workload's own frame count)")
    ap.add_argument("--no-prof", action="store_true")
    ap.add_argument("--shape-table", default=None, help="write the GEMM shape -> tiling table of the profiled step")
    ap.add_argument("--print-losses", action="store_true", help="diagnostic: print every step's loss (host syncs)")
    ap.add_argument("--no-graph", action="store_true",
                    help="launch every kernel from Python each step instead of replaying the captured HIP graph")
    ap.add_argument("--kernel-table", action="store_true",
                    help="after timing, profile one extra step and print per-shape GEMM/attention TF/s to stderr")
    ap.add_argument("--no-trace", action="store_true",
                    help="skip the rocprofv3 kernel-trace run that the roofline's durations come from (N=1)")
    ap.add_argument("--trace-steps", type=int, default=5, help="timed steps of the traced run")
    ap.add_argument("--trace-out", default=None, help="write the traced run's per-kernel CSV here")
    ap.add_argument("--trace-child", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.config == 5:
        args.frames = 16
        if args.dtype is None:
            args.dtype = "fp8"
    if args.dtype is None:
        args.dtype = "bf16"
    return args


# algorithmic flops per profiler record (SURVEY.md §8(d) counting: attention backward = 2 x forward,
# the QK^T recompute of the flash backward is not counted).  V-fold records (m[5] = 1000 + DV: the
# memory cross-attention with its 64-wide value, flash.hip) are priced at the work the fold
# performs: forward 2 (D + DV) per (query, key), backward 2 (2 D + DV) (dP over DV, dQ, dK; no dV)
def record_flops(kind, m):
    if kind == 4:
        b, M, N, K = m[1:5]
        return 2.0 * b * M * N * K
    bh, lq, lk, d = m[1:5]
    if m[5] >= 1000:
        dv = m[5] - 1000
        return 2.0 * bh * lq * lk * ((d + dv) if kind == 1 else (2 * d + dv))
    return (4.0 if kind == 1 else 8.0) * bh * lq * lk * d


def record_bytes(kind, m):
    """algorithmic HBM bytes of one launch: every operand read once, every output written once
    (GEMM: bf16 A, B, C -- fp32 C for weight gradients (layout 4), 1-B A / B for MX-fp8 (layout
    flag 8); attention: Q, K, V, O (+ dO, dQ, dK, dV in the backward), bf16)"""
    if kind == 4:
        b, M, N, K, lay = m[1:6]
        ab = 1 if lay & 8 else 2
        cb = 4 if lay == 4 else 2
        return float(b) * (ab * (M * K + N * K) + cb * M * N)
    bh, lq, lk, d = m[1:5]
    if m[5] >= 1000:  # V-fold: q, k (d wide), memory and u' (dv / dv + 8 wide); backward + dO', dQ, dK
        dv = m[5] - 1000
        fwd = 2.0 * bh * (lq * d + lk * d + lk * dv + lq * (dv + 8))
        return fwd if kind == 1 else 2.0 * fwd
    per = 2.0 * (2 * bh * lq * d + 2 * bh * lk * d)
    return per if kind == 1 else 2.0 * per


FAMILY = {40: "MX-fp8 GEMM (gemm_mx8: forward and dgrad of the projections / FFN, config 5)",
          1: "attention forward (flash_fwd / attn_fwd kernels)",
          2: "attention backward (flash_bwd di/dq/dkv kernels, frame-batched; attn_bwd kernels)",
          4: "GEMM (gemm16g / gemm kernels: projections, FFN, convs, dgrad, wgrad)"}


def family_roofline(recs, nsteps=1):
    """per-family totals of the profiled step(s) (every GEMM / attention launch bracketed by HIP
    events on its own stream; per-step figures = totals / nsteps) and the dominant family (most
    kernel time) as the roofline line"""
    fam = {}
    for ms, m in recs:
        k = 40 if m[0] == 4 and (m[5] & 8) else m[0]  # layout flag 8: MX-fp8 operands
        f = fam.setdefault(k, {"ms": 0.0, "flops": 0.0, "launches": 0, "bytes": 0.0})
        f["ms"] += ms
        f["flops"] += record_flops(m[0], m)
        f["bytes"] += record_bytes(m[0], m)
        f["launches"] += 1
    if not fam:
        return None
    table = {}
    peak = lambda kk: PEAK_FP8_TFLOPS if kk == 40 else PEAK_BF16_TFLOPS  # noqa: E731
    for k, f in fam.items():
        ach = f["flops"] / (f["ms"] * 1e-3) / 1e12 if f["ms"] > 0 else 0.0
        table[FAMILY[k].split(" (")[0]] = {"ms_per_step": round(f["ms"] / nsteps, 3),
                                          "tflop_per_step": round(f["flops"] / nsteps / 1e12, 4),
                                          "achieved": round(ach, 1), "frac": round(ach / peak(k), 4),
                                          "launches_per_step": f["launches"] // nsteps}
    k = max(fam, key=lambda kk: fam[kk]["ms"])
    f = fam[k]
    ach = f["flops"] / (f["ms"] * 1e-3) / 1e12
    return {"bound": "mfma", "achieved": round(ach, 2), "peak": peak(k), "unit": "TFLOP/s",
            "frac": round(ach / peak(k), 4), "traffic": None, "kernel": FAMILY[k],
            "launches": f["launches"], "avg_launch_ms": round(f["ms"] / f["launches"], 4),
            "flops_per_launch_avg": f["flops"] / f["launches"],
            # compare with `traffic` (PMC HBM bytes per launch of the same family)
            "alg_bytes_per_launch": round(f["bytes"] / f["launches"]), "families": table, "_kind": k}


def pmc_traffic(kind):
    """HBM bytes per launch of the dominant family from the newest committed rocprofv3 --pmc
    FETCH_SIZE / WRITE_SIZE passes (profiles/*_<family>_pmc.json, tools/pmc_family.py; counters
    cannot be collected inside this timed run)"""
    import glob
    tag = {1: "attn_fwd", 2: "attn_bwd", 4: "gemm", 40: "gemm_mx8"}[kind]
    import re

    def order(f):  # r<round>_v<version>: numeric, so r02_v16 is newer than r02_v6
        m = re.search(r"r(\d+)_v(\d+)_", os.path.basename(f))
        return (int(m.group(1)), int(m.group(2))) if m else (-1, -1)
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_{tag}_pmc.json")), key=order)
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    return float(d["bytes_per_launch"]), os.path.relpath(files[-1], ROOT)


def read_prof(_lib, with_tags=False):
    """[(ms, [kind, s0..s4])] of every record of the in-library launch profiler (with_tags: a third
    element, the kernel tag of s2h_prof_read_tags)"""
    import ctypes
    n = _lib.lib().s2h_prof_count()
    ms = (ctypes.c_float * max(n, 1))()
    meta = (ctypes.c_int64 * (6 * max(n, 1)))()
    n = _lib.lib().s2h_prof_read(n, ctypes.cast(ms, ctypes.c_void_p), ctypes.cast(meta, ctypes.c_void_p))
    if not with_tags:
        return [(ms[i], [meta[6 * i + j] for j in range(6)]) for i in range(n)]
    tags = (ctypes.c_int64 * max(n, 1))()
    _lib.lib().s2h_prof_read_tags(n, ctypes.cast(tags, ctypes.c_void_p))
    return [(ms[i], [meta[6 * i + j] for j in range(6)], tags[i]) for i in range(n)]


def kernel_name(kind, tag):
    """the kernel a profiler record launched, as rocprofv3 names it (GEMM tilings from the tag of
    s2h_prof_read_tags; attention entry points by family -- one record may span a kernel and its
    key-split combine)"""
    if kind != 4 or not tag:
        return {1: "attention forward entry (flash_fwd / attn_fwd kernels)",
                2: "attention backward entry (flash_bwd kernels)"}.get(kind, "gemm_kernel (fp32)")
    bm, bn = tag & 0x3FF, (tag >> 10) & 0x3FF
    wgm, wgn, ns, bk = (tag >> 20) & 0xF, (tag >> 24) & 0xF, (tag >> 28) & 0xF, 32 * ((tag >> 32) & 0xF)
    akc, bkc, regs, mx8, areg, wgdet, ffn, ffnf = [bool((tag >> b) & 1) for b in (36, 37, 38, 39, 40, 41, 42, 43)]
    tf = lambda x: "true" if x else "false"  # noqa: E731
    if ffn:  # memory-attention FFN backward input gradients in one launch (csrc/ffn.hip)
        return f"(anonymous namespace)::ffn_bwd_dgrad_kernel<{bm}>((anonymous namespace)::FfnArgs)"
    if ffnf:  # memory-attention FFN forward in one launch (csrc/ffn.hip, opt-in)
        return "(anonymous namespace)::ffn_fwd_kernel"
    if wgdet:  # deterministic long-reduction weight gradient (csrc/gemm_wgrad.hip)
        return f"gemm_wg_kernel<{bm}, {bn}, {wgm}, {wgn}, {ns}>"
    if areg:  # short-K tiling with A in registers (gemm_bf16.h gemm16a_kernel, K <= 256)
        return f"gemm16a_kernel<{bn}, 256, {tf(bkc)}>"
    if mx8:
        return f"gemm_mx8_kernel<{bm}, {bn}>"
    if regs:
        return f"gemm16_kernel<{bm}, {bn}, {tf(akc)}, {tf(bkc)}>"
    return f"gemm16g_kernel<{bm}, {bn}, {wgm}, {wgn}, {ns}, {bk}, {tf(akc)}, {tf(bkc)}>"


# kernel-name families of the rocprofv3 trace, matching the in-library profiler's record kinds
TRACE_FAMILY_RX = {4: r"gemm16[ag]?_kernel|gemm16_kernel|gemm_kernel<|gemm_wg|gemm_split|ffn_",
                   40: r"gemm_mx8|mx8_quant",
                   1: r"flash_fwd|flash_combine|attn_fwd|attn_win_fwd",
                   2: r"flash_bwd|attn_bwd|attn_win_bwd|attn_fewq_dkv|attn_fewk_dq"}


def traced_run(args):
    """A child `rocprofv3 --kernel-trace -- python bench.py --trace-child ...` of the same workload
    (started before this process touches the GPU): per-kernel (name, calls, total ms) of the dispatches
    between its trace markers, i.e. its timed graph replays; (rows, steps, note)"""
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3")
    if prof is None:
        return None, 0, "rocprofv3 not found"
    tdir = tempfile.mkdtemp(prefix="s2h_trace_")
    cmd = [prof, "--kernel-trace", "-f", "csv", "-d", tdir, "-o", "kt", "--", sys.executable,
           os.path.abspath(__file__), "--trace-child", "--no-trace", "--no-prof", "--cpu-baseline", "0",
           "--steps", str(args.trace_steps), "--warmup", "2", "--size", args.size, "--image-size",
           str(args.image_size), "--frames", str(args.frames), "--objects", str(args.objects), "--dtype",
           args.dtype, "--config", str(args.config), "--trainable", args.trainable]
    if args.dropout is not None:
        cmd += ["--dropout", str(args.dropout)]
    try:
        r = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, timeout=420)
        if r.returncode != 0:
            return None, 0, f"traced run exited {r.returncode}: {r.stderr.decode(errors='replace')[-300:]}"
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import step_profile
        rows = step_profile.load_region(tdir, verbose=False)
        if not rows:
            return None, 0, "no kernel trace written"
        if args.trace_out:
            step_profile.write_stats(rows, args.trace_steps, args.trace_out)
        return rows, args.trace_steps, "ok"
    except Exception as e:  # the trace refines the roofline; it is never required
        return None, 0, f"trace failed: {e!r}"
    finally:
        shutil.rmtree(tdir, ignore_errors=True)


def trace_roofline(rows, tsteps, recs3, kind_hint=None):
    """The roofline from the kernel trace of the timed replays: per family, the algorithmic flops of
    one step (the in-library profiler's records of the profiled eager step: shapes only, its event
    times unused) over the family's kernel time per step in the trace; the dominant family is the one
    with the most traced time, its dominant kernel the traced kernel with the most time, priced with
    the flops per launch of the records that launched that kernel (bench.kernel_name of their tags)."""
    import re
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import step_profile
    fam_ms, fam_calls = {}, {}
    per_name = {}
    for name, calls, ms in rows:
        sn = step_profile.short(name)
        per_name[sn] = (calls, ms)
        for k, rx in TRACE_FAMILY_RX.items():
            if re.search(rx, name):
                fam_ms[k] = fam_ms.get(k, 0.0) + ms / tsteps
                fam_calls[k] = fam_calls.get(k, 0) + calls / tsteps
                break
    fl, by, names = {}, {}, {}
    for ms, m, tag in recs3:
        k = 40 if m[0] == 4 and (m[5] & 8) else m[0]
        fl[k] = fl.get(k, 0.0) + record_flops(m[0], m)
        by[k] = by.get(k, 0.0) + record_bytes(m[0], m)
        a = names.setdefault(kernel_name(m[0], tag), [0, 0.0, 0.0])
        a[0] += 1
        a[1] += record_flops(m[0], m)
        a[2] += record_bytes(m[0], m)
    if not fam_ms or not fl:
        return None
    peak = lambda kk: PEAK_FP8_TFLOPS if kk == 40 else PEAK_BF16_TFLOPS  # noqa: E731
    table = {}
    for k in fam_ms:
        if k not in fl:
            continue
        ach = fl[k] / (fam_ms[k] * 1e-3) / 1e12
        table[FAMILY[k].split(" (")[0]] = {"ms_per_step": round(fam_ms[k], 3), "tflop_per_step": round(fl[k] / 1e12, 4),
                                          "achieved": round(ach, 1), "frac": round(ach / peak(k), 4),
                                          "kernels_per_step": round(fam_calls[k], 1)}
    k = kind_hint if kind_hint in fam_ms and kind_hint in fl else max((kk for kk in fam_ms if kk in fl),
                                                                      key=lambda kk: fam_ms[kk])
    ach = fl[k] / (fam_ms[k] * 1e-3) / 1e12
    out = {"bound": "mfma", "achieved": round(ach, 2), "peak": peak(k), "unit": "TFLOP/s", "frac": round(ach / peak(k), 4),
           "kernel": FAMILY[k], "kernels_per_step": round(fam_calls[k], 1), "ms_per_step": round(fam_ms[k], 3),
           "alg_flop_per_step": fl[k], "alg_bytes_per_step": by[k], "families": table, "_kind": k}
    # dominant kernel: the family's traced kernel with the most time that the profiler records name
    cands = [(n, c, ms) for n, (c, ms) in per_name.items() if n in names
             and re.search(TRACE_FAMILY_RX[k], n)]
    if cands:
        n, c, ms = max(cands, key=lambda r: r[2])
        rn, rfl, rby = names[n]
        avg_us = 1e3 * ms / c
        a = rfl / rn / (avg_us * 1e-6) / 1e12
        out["dominant_kernel"] = {"name": n, "launches_per_step": round(c / tsteps, 1), "avg_us": round(avg_us, 2),
                                  "alg_flop_per_launch": round(rfl / rn), "alg_bytes_per_launch": round(rby / rn),
                                  "achieved_tflops": round(a, 1), "frac": round(a / peak(k), 4),
                                  "share_of_family_ms": round(ms / tsteps / fam_ms[k], 3),
                                  "profiled_launches_per_step": rn}
    return out


def event_overhead_ms(_lib, n=64):
    """Per-record overhead of the in-library event brackets: `n` empty kernels (s2h_trace_marker)
    each bracketed like a profiled launch, minus the per-kernel time of `n` back-to-back empty
    kernels between one event pair (their execution + dispatch, as a replayed graph sees it).
    An eager launch bracketed by events also times the dispatch ramp in front of the kernel; this
    is subtracted from the dominant kernel's average so it is comparable with rocprofv3's
    start-to-end kernel durations."""
    st = torch.cuda.current_stream()
    _lib.call("s2h_prof_reset")
    _lib.call("s2h_prof_select", 8)
    for _ in range(n):
        _lib.call("s2h_trace_marker", 0, st.cuda_stream)
    torch.cuda.synchronize()
    bracketed = sorted(ms for ms, m in read_prof(_lib) if m[0] == 8)
    _lib.call("s2h_prof_select", 0)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(n):
        _lib.call("s2h_trace_marker", 0, st.cuda_stream)
    e1.record(st)
    torch.cuda.synchronize()
    burst = e0.elapsed_time(e1) / n
    _lib.call("s2h_prof_reset")
    return max(0.0, bracketed[len(bracketed) // 2] - burst), bracketed[len(bracketed) // 2], burst


def dominant_kernel(recs, kind, peak, nsteps=1, overhead_ms=0.0):
    """the single kernel with the most time in family `kind` (records tagged with the GEMM tiling
    they launched): launches and avg duration per launch, algorithmic flop / bytes per launch (the
    family's pricing), achieved rate and fraction of peak -- traceable to the same kernel's row of
    a rocprofv3 kernel-stats summary"""
    agg = {}
    for ms, m, tag in recs:
        k = 40 if m[0] == 4 and (m[5] & 8) else m[0]
        if k != kind:
            continue
        a = agg.setdefault(kernel_name(m[0], tag), [0, 0.0, 0.0, 0.0])
        a[0] += 1
        a[1] += ms
        a[2] += record_flops(m[0], m)
        a[3] += record_bytes(m[0], m)
    if not agg:
        return None
    name, (n, ms, fl, by) = max(agg.items(), key=lambda kv: kv[1][1] - kv[1][0] * overhead_ms)
    raw = ms / n
    avg = max(raw - overhead_ms, 1e-6)  # event-bracket overhead removed (event_overhead_ms)
    ach = fl / n / (avg * 1e-3) / 1e12
    return {"name": name, "launches_per_step": n // nsteps, "avg_us": round(1e3 * avg, 2),
            "avg_us_event_bracket": round(1e3 * raw, 2), "event_overhead_us": round(1e3 * overhead_ms, 2),
            "alg_flop_per_launch": round(fl / n), "alg_bytes_per_launch": round(by / n),
            "achieved_tflops": round(ach, 1), "frac": round(ach / peak, 4),
            "share_of_family_ms": None}


def write_shape_table(recs3, path):
    """GEMM shape -> tiling table of one profiled eager step: for every (tiling kernel, shape, operand
    layout) its launches per step and algorithmic flops per launch (so a traced kernel's flops per
    launch -- the roofline's dominant kernel -- can be recomputed shape by shape), and the event-bracketed
    time per launch (overstates short launches by the event overhead; the trace is the time reference)"""
    agg = {}
    for ms, m, tag in recs3:
        if m[0] != 4:
            continue
        b, M, N, K, lay = m[1:]
        key = (kernel_name(4, tag), f"b{b} {M}x{N}x{K} {'A' if lay & 2 else 'a'}{'B' if lay & 1 else 'b'}")
        a = agg.setdefault(key, [0, 0.0, record_flops(4, m)])
        a[0] += 1
        a[1] += ms
    by_kernel = {}
    for (kn, shape), (n, ms, fl) in agg.items():
        by_kernel.setdefault(kn, []).append((shape, n, fl, ms))
    with open(path, "w") as f:
        f.write("# GEMM shape -> tiling of one profiled eager step (bench.py --shape-table): kernel | shape (batch MxNxK,\n"
                "# A/a = A K-contiguous or not, B/b likewise) | launches | GFLOP per launch | event us per launch\n")
        for kn, rows in sorted(by_kernel.items(), key=lambda kv: -sum(r[1] * r[2] for r in kv[1])):
            n_all = sum(r[1] for r in rows)
            fl_all = sum(r[1] * r[2] for r in rows)
            f.write(f"\n{kn}: {n_all} launches, {fl_all / max(n_all, 1) / 1e9:.3f} GFLOP per launch on average\n")
            for shape, n, fl, ms in sorted(rows, key=lambda r: -r[1] * r[2]):
                f.write(f"  {shape:32s} n={n:4d}  {fl / 1e9:8.3f} GF  {1e3 * ms / n:8.2f} us\n")


def kernel_table(recs):
    """Per-shape time / achieved TFLOP/s of the GEMM and attention launches of one step."""
    agg = {}
    for ms, m in recs:
        kind = m[0]
        if kind == 4:
            b, M, N, K, lay = m[1:]
            key = ("gemm_mx8" if lay & 8 else "gemm",
                   f"b{b} {M}x{N}x{K} {'AB'[0] if lay & 2 else 'a'}{'B' if lay & 1 else 'b'}")
            fl = 2.0 * b * M * N * K
        else:
            bh, lq, lk, d, tag = m[1:]
            if tag >= 1000:  # V-fold (executed work incl. the backward's QK^T recompute)
                dv = tag - 1000
                key = ("attn_fwd" if kind == 1 else "attn_bwd", f"bh{bh} {lq}x{lk} d{d} vfold{dv}")
                fl = 2.0 * bh * lq * lk * ((d + dv) if kind == 1 else (3 * d + dv))
            else:
                key = ("attn_fwd" if kind == 1 else "attn_bwd", f"bh{bh} {lq}x{lk} d{d}")
                fl = (4.0 if kind == 1 else 10.0) * bh * lq * lk * d
        a = agg.setdefault(key, [0, 0.0, 0.0])
        a[0] += 1
        a[1] += ms
        a[2] += fl
    rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
    tot = sum(v[1] for v in agg.values())
    out = [f"# profiled step: {tot:.2f} ms in GEMM + attention launches"]
    for (kind, shape), (n, ms, fl) in rows:
        out.append(f"{kind:9s} {shape:34s} n={n:4d} {ms:8.3f} ms {fl / (ms * 1e-3) / 1e12:7.1f} TF/s")
    return "\n".join(out)


def cpu_baseline(args):
    """CPU oracle (oracle/sam2_oracle.py, fp32 PyTorch-CPU restatement of the reference step)
    on a bounded sample: one clip of the same shape with `cpu_frames` frames, fwd+loss+bwd."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import sam2_oracle as O
    from sam2_video.data.synthetic import make_clip
    from sam2_video.model.configs import model_config
    from sam2_video.utils.init import synth_tensor

    # the host's CPU share: OMP_NUM_THREADS (16 per GPU on the GPU box) when set, else every core
    threads = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
    torch.set_num_threads(threads)
    frames = args.cpu_frames or args.frames
    cfg = model_config(args.size, args.image_size)
    trainable = ALL if args.trainable == "all" else ["memory_attention", "memory_encoder"]
    P = O.make_params(O.param_shapes(cfg), O.trainable_prefixes(trainable), synth_tensor, seed=0)
    clip = make_clip(10_000, frames, args.image_size, args.objects, args.objects)
    model = O.OracleSAM2(cfg, P, dropout=0.0)
    t0 = time.time()
    stages, merged, aux = model.forward(clip["images"], clip["masks"])
    losses = O.multistep_loss(merged, clip["masks"])
    losses["total_loss"].backward()
    dt = time.time() - t0
    return {"value": round(frames / dt, 4), "unit": "clip-frames/s", "cores": threads, "kind": "port",
            "sample": f"1 clip x {frames} frames (the timed workload's clip), {args.size} {args.image_size}^2, "
                      f"{args.objects} objects, fp32 fwd+loss+bwd (oracle, no optimizer step), {dt:.1f} s, "
                      f"{threads} threads"}


def spawn_ranks(n):
    """`bench.py --gpus N` outside torchrun: start N rank processes (one per GPU, RCCL over
    127.0.0.1) before this parent touches the GPU, wait for all, exit with the worst status.
    Rank 0 prints the JSON line."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    codes = [p.wait() for p in procs]
    return max(codes, key=abs)


def main():
    args = parse()
    if args.gpus > 1 and "RANK" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    trace = (None, 0, "off")
    under_profiler = any(k.startswith("ROCPROF") for k in os.environ)  # never nest a traced run in one
    if (not args.no_trace and not args.trace_child and not args.no_prof and args.gpus == 1 and not under_profiler
            and os.environ.get("WORLD_SIZE", "1") == "1"):
        trace = traced_run(args)  # before this process initialises the GPU
    from sam2_video.data.synthetic import make_clip, sam2_collate_fn
    from sam2_video.kernels import _lib
    from sam2_video.kernels import functional as FN
    from sam2_video.model.sam2model import SAM2Model
    from sam2_video.training.ddp import init_from_env, shard_clips
    from sam2_video.training.trainer import SAM2LightningModule, StepRunner

    # S2H_DIST_BACKEND=gloo: rehearsal of the N > 1 path with several ranks sharing the GPUs there
    # are (rank -> GPU local % count), e.g. 2 ranks on a 1-GPU box; the scaling runs use RCCL
    backend = os.environ.get("S2H_DIST_BACKEND", "nccl")
    rank, world, local = init_from_env(backend)
    dev = local if backend == "nccl" else local % max(1, torch.cuda.device_count())
    if world == 1 or backend != "nccl":
        torch.cuda.set_device(dev)
    device = torch.device("cuda", dev)
    FN.set_seed(1234 + rank)
    trainable = ALL if args.trainable == "all" else ["memory_attention", "memory_encoder"]
    model = SAM2Model(None, f"{args.size}@{args.image_size}", trainable_modules=trainable, compute_dtype=args.dtype)
    if args.dropout is not None:
        model.set_dropout(args.dropout)
    loss_cfg = {"type": "multi_step", "gt_stride": 1, "multistep_logit_temperature": 1.0,
                "weight_dict": {"loss_mask": 20, "loss_dice": 1, "loss_iou": 1, "loss_class": 0},
                "supervise_all_iou": True, "iou_use_l1_loss": True, "pred_obj_scores": False,
                "focal_gamma_obj_score": 0.0, "focal_alpha_obj_score": -1.0}
    opt_cfg = {"type": "AdamW", "lr": 4e-6, "weight_decay": 0.01, "betas": [0.9, 0.999], "warmup_factor": 0.15}
    module = SAM2LightningModule(model, loss_cfg, opt_cfg, {"enabled": True, "num_cycles": 0.5})
    module.setup("fit", device)
    total = args.warmup + args.steps
    graph = not args.no_graph
    runner = StepRunner(module, total_steps=total, distributed=world > 1, graph=graph)

    # synthetic clips, resident in HBM before timing (clip index = rank + k * world)
    batches = []
    for idx in shard_clips(total, rank, world):
        clip = make_clip(idx, args.frames, args.image_size, args.objects, args.objects)
        batches.append(sam2_collate_fn([clip]).to(device))
    torch.cuda.synchronize()

    for k in range(args.warmup):
        loss = runner(batches[k])
        if args.print_losses:
            print(f"step {k} loss {float(loss):.5f}", file=sys.stderr)
    torch.cuda.synchronize()
    if not args.no_prof and not graph:
        _lib.call("s2h_prof_enable", 16384)
        _lib.call("s2h_prof_select", 7)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # trace markers: a rocprofv3 kernel trace of this run keeps exactly the timed steps between them
    # (tools/step_profile.py; no setup copies, warm-up or profiled eager step)
    _lib.call("s2h_trace_marker", 1, torch.cuda.current_stream().cuda_stream)
    t0 = time.perf_counter()
    for k in range(args.warmup, total):
        loss = runner(batches[k])
        if args.print_losses:
            fr = " ".join(f"{float(f['multistep_pred_multimasks_high_res'][0].abs().mean()):.3g}"
                          f"/{float(f['multistep_pred_ious'][0].abs().mean()):.3g}" for f in module.last_outputs)
            print(f"step {k} loss {float(loss):.5f} graphs {len(runner._graphs)} frames {fr}", file=sys.stderr)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    _lib.call("s2h_trace_marker", 2, torch.cuda.current_stream().cuda_stream)
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    loss_val = float(module.logged["train/total_loss"])  # last timed step
    if not math.isfinite(loss_val):
        print(f"ERROR: non-finite training loss {loss_val} in the timed steps", file=sys.stderr)
        sys.exit(3)
    roof = None
    if not args.no_prof:
        if graph:
            # HIP events cannot time kernels inside a replayed graph (ROCm 7.2 rejects external
            # event nodes in capture): time the same kernels in one eager step right after the
            # timed region, each launch bracketed by events on its own stream
            _lib.call("s2h_prof_enable", 16384)
            _lib.call("s2h_prof_select", 7)
            runner.graph = False
            runner(batches[-1])
            runner.graph = True
            torch.cuda.synchronize()
            print(f"profiled eager step loss {float(module.logged['train/total_loss']):.5f}", file=sys.stderr)
        recs3 = read_prof(_lib, with_tags=True)
        recs = [(ms, m) for ms, m, _ in recs3]
        ovh, ev_empty, burst = event_overhead_ms(_lib)  # (profiler still on: bracketed empty launches)
        _lib.call("s2h_prof_enable", 0)
        nsteps = 1 if graph else args.steps
        roof = family_roofline(recs, nsteps)
        if roof is not None:
            kind = roof.pop("_kind")
            dk = dominant_kernel(recs3, kind, roof["peak"], nsteps, ovh)
            if dk is not None:
                fam_ms = roof["avg_launch_ms"] * roof["launches"]
                dk["share_of_family_ms"] = round(dk["avg_us_event_bracket"] * 1e-3 * dk["launches_per_step"] * nsteps
                                                 / fam_ms, 3)
                dk["event_calibration"] = (f"empty kernel: {1e3 * ev_empty:.2f} us event-bracketed, {1e3 * burst:.2f} us "
                                           "per kernel back to back; the difference is subtracted")
            roof["dominant_kernel"] = dk
            roof["traffic"], src = pmc_traffic(kind)
            if src:
                roof["traffic_unit"] = "HBM bytes per launch (2*FETCH_SIZE + WRITE_SIZE), same launch mix"
                roof["traffic_source"] = src
            roof["timing"] = ("HIP events per launch, one eager step after the timed graph replays" if graph
                              else "HIP events per launch over the timed region")
            rows, tsteps, note = trace
            troof = trace_roofline(rows, tsteps, recs3) if rows else None
            if troof is not None:
                # the trace drives bound / achieved / frac / dominant_kernel; the event-bracketed figures
                # stay beside them for comparison
                troof.pop("_kind")
                ev = {k: roof[k] for k in ("kernel", "achieved", "frac", "launches", "avg_launch_ms", "families",
                                          "dominant_kernel", "timing") if k in roof}
                for k in ("traffic", "traffic_unit", "traffic_source", "alg_bytes_per_launch"):
                    if k in roof:
                        troof[k] = roof[k]
                troof["timing"] = (f"rocprofv3 kernel trace of the {tsteps} timed graph replays of a traced run of "
                                   "this workload (bench.py --trace-child, started before the timed run); flops "
                                   "per launch from the in-library profiler's records of one eager step")
                troof["event_based"] = ev
                roof = troof
            else:
                roof["trace"] = note
        if args.kernel_table and rank == 0:
            print(kernel_table(recs), file=sys.stderr, flush=True)
        if args.shape_table and rank == 0:
            write_shape_table(recs3, args.shape_table)
        _lib.call("s2h_prof_select", 1)

    frames = args.frames * args.steps * world
    value = frames / elapsed
    if args.trace_child:  # the traced run only supplies the kernel trace of its timed replays
        return

    # validation IoU (eval/eval.py formulas, in-loop) on a held-out synthetic clip per rank
    val_clip = make_clip(100_000 + rank, args.frames, args.image_size, args.objects, args.objects)
    module.validation_step(sam2_collate_fn([val_clip]).to(device))
    val_iou = float(module.last_eval["avg_scores"]["iou"])
    if world > 1:
        t = torch.tensor([val_iou], device=device)
        dist.all_reduce(t)
        val_iou = float(t.item()) / world
    result = {
        "metric": "training clip-frames/sec (512^2 8-frame, Hiera-B+)",
        "value": round(value, 3),
        "unit": "clip-frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 2),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype if args.dtype != "fp8" else "fp8 (MX e4m3 fwd + dgrad of projections / FFN) + bf16",
        "data": "synthetic (N(0,1) images, drifting disc masks; deterministic synthetic weights, no checkpoint)",
        "config": {"workload": f"SAM2 video fine-tuning step, sam2.1_hiera_{args.size}, {args.image_size}^2, "
                               f"{args.frames} frames, {args.objects} objects, trainable={args.trainable}",
                   "global_batch": world, "clips_per_rank": 1, "frames": args.frames,
                   "image_size": args.image_size, "objects": args.objects, "parallelism": f"dp{world}"},
        "roofline": roof,
        # whole-step MFMA utilisation: algorithmic TF per clip-frame x rate / peak
        "step_mfma_frac": (round(STEP_TF_PER_FRAME[(args.size, args.image_size, args.frames, args.objects, args.trainable)] * value
                                 / (PEAK_BF16_TFLOPS * world), 4)
                           if (args.size, args.image_size, args.frames, args.objects, args.trainable) in STEP_TF_PER_FRAME else None),
        "cpu_baseline": None,
        "final_loss": round(loss_val, 5),
        # eval.py IoU of the category-merged masks on held-out synthetic clips (random-init weights
        # after `steps` fine-tuning steps: a pipeline check, not a model-quality number)
        "val_iou": round(val_iou, 5),
    }
    if rank == 0 and world == 1 and args.cpu_baseline:
        try:
            result["cpu_baseline"] = cpu_baseline(args)
        except Exception as e:  # the baseline is reported, never required
            result["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
