"""Packed-fp32 hazard scan of the library's device code.

Round 4 traced intermittently wrong results in the RoPE GEMM epilogue to packed-fp32 VALU pairs
(v_pk_mul_f32 / v_pk_fma_f32 with cross-half op_sel) where an instruction overwrote a register the
packed instruction right before it still read; the library is built with -fno-slp-vectorize since.
Explicit vector code can still compile to packed fp32 ops.  This compiles every csrc/*.hip to gfx950
assembly and reports, per kernel, the packed-fp32 instructions and every one of them whose register
sources are overwritten by one of the next `--window` VALU instructions (the round-4 pattern).

    python tools/pk_f32_scan.py [--window 2] [--keep DIR]      (CPU only: hipcc cross-compiles)"""
import argparse
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "sam2-video-training_amd", "csrc")
PK = re.compile(r"^\s*(v_pk_(?:mul|fma|add)_f32)\s+(.*)$")
VALU = re.compile(r"^\s*(v_[a-z0-9_]+)\s+(.*)$")
REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def operands(rest):
    parts = [p.strip() for p in re.split(r",(?![^\[]*\])", rest.split(" op_sel")[0].split(" neg_")[0])]
    return parts[0], parts[1:]


def scan(asm, window):
    per_kernel = collections.Counter()
    hazards = []
    fn = None
    lines = open(asm).read().splitlines()
    for i, ln in enumerate(lines):
        lm = re.match(r"^([A-Za-z_][\w.$]*):", ln)
        if lm:
            fn = lm.group(1)
        m = PK.match(ln)
        if not m:
            continue
        per_kernel[fn] += 1
        _, srcs = operands(m.group(2))
        src_regs = set().union(*(regs(s) for s in srcs)) if srcs else set()
        seen = 0
        for j in range(i + 1, min(len(lines), i + 40)):
            v = VALU.match(lines[j])
            if not v or v.group(1).startswith(("v_mfma", "v_readfirstlane", "v_readlane")):
                continue
            dst, _ = operands(v.group(2))
            if regs(dst) & src_regs:
                hazards.append((fn, i + 1, ln.strip(), lines[j].strip()))
                break
            seen += 1
            if seen >= window:
                break
    return per_kernel, hazards


def makefile_flags():
    """the library's CXXFLAGS (csrc/Makefile), continuation lines joined"""
    text = open(os.path.join(CSRC, "Makefile")).read().replace("\\\n", " ")
    line = next(ln for ln in text.splitlines() if ln.startswith("CXXFLAGS"))
    return [f.replace("$(ARCH)", "gfx950") for f in line.split("=", 1)[1].split() if f not in ("-fPIC",)]


FLAGS = makefile_flags()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--window", type=int, default=2)
    ap.add_argument("--keep", default=None)
    args = ap.parse_args()
    out = args.keep or tempfile.mkdtemp()
    os.makedirs(out, exist_ok=True)
    srcs = sorted(f for f in os.listdir(CSRC) if f.endswith(".hip"))
    procs = []
    for f in srcs:
        procs.append(subprocess.Popen(["/opt/rocm/bin/hipcc"] + FLAGS + ["--cuda-device-only", "-S", "-o",
                                       os.path.join(out, f[:-4] + ".s"), f], cwd=CSRC, stderr=subprocess.DEVNULL))
    for p in procs:
        p.wait()
    total_h = 0
    for f in srcs:
        pk, hz = scan(os.path.join(out, f[:-4] + ".s"), args.window)
        if pk:
            print(f"{f}: {sum(pk.values())} packed-fp32 instructions in {len(pk)} kernels, {len(hz)} flagged")
            for fn, n in pk.most_common():
                print(f"    {n:5d}  {fn[:110]}")
        for fn, line, a, b in hz:
            print(f"    HAZARD {fn[:80]} line {line}: {a}  ->  {b}")
        total_h += len(hz)
    print(f"flagged pairs: {total_h}")
    sys.exit(1 if total_h else 0)


if __name__ == "__main__":
    main()
