"""Extract glibc's powf tables from this image's libm.so.6 and emit
raytracingtherestofyourlife_amd/csrc/glibc_powf.hpp's data block.

vtkm::Pow(float, float) is std::pow -> powf on the reference's CPU build
(RayTracer SurfaceColor::Shade, the -direct colour mode: pow(max(cosPhi,0), 20)).
glibc 2.35's powf (sysdeps/ieee754/flt-32/e_powf.c) is not correctly rounded,
so the device restates its algorithm with glibc's own tables:
  __powf_log2_data: 16 x {invc, logc} + poly[5]      (powf_log2_data.c)
  __exp2f_data:     tab[32] (uint64), shift_scaled, poly[3]  (exp2f_data.c)
The tables are internal symbols, located here by structure (a run of 16
(invc, log2(1/invc)) pairs followed by the powf log2 polynomial, and the exp2
table that starts with 1.0 and asuint64(2^(1/32)) - (1 << 47)), then printed
as hex constants.  tests/test_direct.py re-checks the committed header against
libm (the constants and, exhaustively over [0, 1.01] for y = 20, the results).

usage: python tools/extract_glibc_powf.py [libm path]  (prints the C++ block)
"""
from __future__ import annotations

import math
import struct
import sys

LIBM = "/lib/x86_64-linux-gnu/libm.so.6"


def locate(data: bytes):
    t1 = struct.unpack("<Q", struct.pack("<d", 2 ** (1 / 32)))[0] - (1 << 47)
    exp2 = data.find(struct.pack("<QQ", 0x3FF0000000000000, t1))
    if exp2 < 0:
        raise RuntimeError("exp2f table not found")

    def pairs16(off):
        for k in range(16):
            invc, logc = struct.unpack_from("<dd", data, off + 16 * k)
            if not (0.6 < invc < 1.6) or not math.isfinite(logc) or abs(logc - math.log2(1 / invc)) > 1e-6:
                return False
        return True

    log2 = -1
    for off in range(0, len(data) - 512, 8):
        if pairs16(off):
            poly = struct.unpack_from("<5d", data, off + 256)
            # the powf log2 polynomial approximates log1p(r)/ln2: last coefficient ~ 1/ln2, 5 terms
            if abs(poly[4] - 1 / math.log(2)) < 1e-6 and abs(poly[3] + 0.5 / math.log(2)) < 1e-3:
                log2 = off
                break
    if log2 < 0:
        raise RuntimeError("powf log2 table not found")
    return log2, exp2


def tables(path: str = LIBM):
    data = open(path, "rb").read()
    log2, exp2 = locate(data)
    log2_tab = struct.unpack_from("<32Q", data, log2)
    log2_poly = struct.unpack_from("<5Q", data, log2 + 256)
    exp2_tab = struct.unpack_from("<32Q", data, exp2)
    shift_scaled, c0, c1, c2 = struct.unpack_from("<4Q", data, exp2 + 256)
    return {"log2_tab": log2_tab, "log2_poly": log2_poly, "exp2_tab": exp2_tab,
            "exp2_shift_scaled": shift_scaled, "exp2_poly": (c0, c1, c2)}


def emit(t) -> str:
    def arr(name, vals, per=4):
        rows = [", ".join(f"0x{v:016x}ull" for v in vals[i:i + per]) for i in range(0, len(vals), per)]
        return f"constexpr uint64_t {name}[{len(vals)}] = {{\n    " + ",\n    ".join(rows) + "};\n"
    return (arr("kPowfLog2Tab", t["log2_tab"]) + arr("kPowfLog2Poly", t["log2_poly"], 5)
            + arr("kExp2fTab", t["exp2_tab"])
            + f"constexpr uint64_t kExp2fShiftScaled = 0x{t['exp2_shift_scaled']:016x}ull;\n"
            + arr("kExp2fPoly", t["exp2_poly"], 3))


if __name__ == "__main__":
    print(emit(tables(sys.argv[1] if len(sys.argv) > 1 else LIBM)))
