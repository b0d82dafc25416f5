"""Static VALU attribution of one kernel's ISA (development tool, CPU only).

Compiles rtp_kernels.hip for gfx950 to assembly with line tables, cuts out one
kernel, and counts its vector instructions per source line (the innermost
inlined location of each instruction) and per basic block.  Static counts:
how often a block runs is not known here, but the per-region totals of the
straight-line parts of a bounce (quad tests, generator, pdfs) are the VALU
instructions one bounce step issues there.

usage: python tools/isa_attrib.py [--kernel SUBSTR] [--defines="-DX=1 ..."] [--top N] [--blocks]
"""
from __future__ import annotations

import argparse
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "raytracingtherestofyourlife_amd", "csrc")


def compile_asm(out: str, defines: list[str]) -> None:
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-fno-slp-vectorize",
           "--cuda-device-only", "-S", "-gline-tables-only", *defines, "-o", out,
           os.path.join(CSRC, "rtp_kernels.hip"), f"-I{CSRC}"]
    subprocess.run(cmd, check=True, capture_output=True)


def kernel_lines(asm: str, substr: str) -> list[str]:
    lines = open(asm).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and substr in l.split(":")[0])
    end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
    files = {}
    for l in lines:
        m = re.match(r'\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', l)
        if m:
            files[int(m.group(1))] = os.path.basename(m.group(2))
    return lines[start:end + 1], files


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="rtp_render_poolILb0ELb0ELb1E")
    ap.add_argument("--defines", default="", help='e.g. --defines="-DRTP_X=0 -DRTP_Y=1"')
    ap.add_argument("--asm", default="/tmp/rtp_isa.s")
    ap.add_argument("--no-compile", action="store_true")
    ap.add_argument("--top", type=int, default=60)
    ap.add_argument("--blocks", action="store_true")
    a = ap.parse_args()
    if not a.no_compile:
        compile_asm(a.asm, a.defines.split())
    body, files = kernel_lines(a.asm, a.kernel)
    loc = ("?", 0)
    per_line = collections.Counter()
    per_block = collections.OrderedDict()
    block = "entry"
    per_block[block] = [0, 0, collections.Counter()]
    kinds = collections.Counter()
    for l in body:
        m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
        if m:
            loc = (files.get(int(m.group(1)), "?"), int(m.group(2)))
            continue
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            block = m.group(1)
            per_block[block] = [0, 0, collections.Counter()]
            continue
        m = re.match(r"\s+(v_\S+|s_\S+|ds_\S+|global_\S+|buffer_\S+|scratch_\S+|flat_\S+)", l)
        if not m:
            continue
        op = m.group(1)
        if op.startswith("v_"):
            per_line[loc] += 1
            per_block[block][0] += 1
            per_block[block][2][loc] += 1
            kinds[op] += 1
        else:
            per_block[block][1] += 1
    total = sum(per_line.values())
    print(f"kernel {a.kernel}: {total} VALU instructions (static)")
    for (f, ln), c in per_line.most_common(a.top):
        print(f"{c:6d}  {f}:{ln}")
    if a.blocks:
        print("\nblocks (VALU, other, top lines):")
        for b, (v, s, locs) in per_block.items():
            top = ", ".join(f"{f}:{ln}x{c}" for (f, ln), c in locs.most_common(4))
            print(f"{b:14s} {v:5d} {s:5d}  {top}")
    print("\nmost frequent VALU opcodes:")
    for op, c in kinds.most_common(25):
        print(f"{c:6d} {op}")


if __name__ == "__main__":
    sys.exit(main())
