"""Build librtp.so (HIP kernels + C ABI) in-tree for gfx950 with hipcc.

The shared object lands next to this file so it travels to the GPU box with
the repository snapshot.  Flags that the parity contract depends on:
  -ffp-contract=off      no a*b+c -> fma contraction (the reference's x86-64
                         g++ build has no FMA);
  no -ffast-math, HIP's default correctly-rounded f32 div/sqrt, denormals kept.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "librtp.so")
SOURCES = ["rtp_kernels.hip", "rtp_direct.hip", "rtp_bvh_gpu.hip", "rtp_host.cpp", "rtp_direct_host.cpp", "scene_cornell.cpp"]
HEADERS = ["rtp_device.hpp", "rtp_layout.hpp", "rtp_context.hpp", "glibc_powf.hpp", os.path.join("..", "..", "include", "rtp.h")]
ARCH = os.environ.get("RTP_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: librtp.so cannot be built")


def flags() -> list[str]:
    # -fno-slp-vectorize: the SLP vectorizer paired scalar float products
    # (dot products, cross products) into v_pk_mul_f32 / v_pk_add_f32, each
    # followed by an s_nop before its result is read (gfx950's packed-FP32
    # hazard); scalar they need none.  C2 101.5-102.9 -> 96.2-97.2 ms (-5.5%),
    # C3 -3.2% (profiles/r04n_ab_noslp.txt).  The explicit packed pairs of the
    # quad tests (ext_vector_type) stay packed.  Results are the same bits:
    # a packed half rounds like the scalar instruction.
    return ["-O3", f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
            "-fno-fast-math", "-fno-slp-vectorize", "-Wall", "-Wno-unused-function", "-Wno-unused-variable"]


def stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.abspath(__file__)]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not stale():
        return LIB
    cmd = [hipcc(), *flags(), "-o", LIB + ".tmp", *[os.path.join(CSRC, s) for s in SOURCES]]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"hipcc failed ({res.returncode}):\n{res.stdout}\n{res.stderr}")
    os.replace(LIB + ".tmp", LIB)
    return LIB


ROOT = os.path.dirname(HERE)
# C++ host programs over the C ABI (include/rtp/rendering.hpp), linked with g++
CPP_PROGRAMS = {
    os.path.join(ROOT, "examples", "rtp_path"): os.path.join(ROOT, "examples", "path_main.cpp"),
    os.path.join(ROOT, "tests", "cpp", "shim_check"): os.path.join(ROOT, "tests", "cpp", "shim_check.cpp"),
}


def build_cpp(force: bool = False) -> list[str]:
    """g++ the C++ host programs against librtp.so (rpath to the package dir)."""
    lib = build()
    built = []
    hdrs = [os.path.join(ROOT, "include", "rtp.h"), os.path.join(ROOT, "include", "rtp", "rendering.hpp"), lib]
    for exe, src in CPP_PROGRAMS.items():
        rel = os.path.relpath(HERE, os.path.dirname(exe))
        if force or not os.path.exists(exe) or any(os.path.getmtime(d) > os.path.getmtime(exe) for d in hdrs + [src]):
            cmd = [os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-Wall", "-I", os.path.join(ROOT, "include"), src,
                   "-L", HERE, "-lrtp", f"-Wl,-rpath,$ORIGIN/{rel}", "-o", exe]
            res = subprocess.run(cmd, capture_output=True, text=True)
            if res.returncode != 0:
                raise RuntimeError(f"g++ failed for {src}:\n{res.stderr}")
        built.append(exe)
    return built


# The reference's own main.cc and CornellBox.cpp, compiled UNCHANGED against
# librtp.so through the VTK-m-named headers of include/vtkm_compat
# (rtp/vtkm_compat.hpp): each read from its place in the reference tree on
# stdin, so that its quoted includes ("MapperPathTracer.h", "View3D.h",
# "pathtracing/SphereExtractor.h", ...) resolve in include/vtkm_compat/ (the
# compile's working directory) first; "CornellBox.h" and the
# "pathtracing/vec3.h" it includes are the reference's own (-iquote).
# Nothing of the reference is copied; the binaries are built where the
# reference exists (this container) and travel to the GPU box like librtp.so.
REFERENCE_DIR = os.environ.get("RTP_REFERENCE_DIR", "/root/reference")
REFERENCE_MAIN = os.path.join(REFERENCE_DIR, "main.cc")
REFERENCE_SOURCES = ("main.cc", "CornellBox.cpp")
MAIN_UNCHANGED = os.path.join(ROOT, "examples", "main_cc")
SCENE_CHECK = os.path.join(ROOT, "tests", "cpp", "scene_unchanged_check")


def build_main_unchanged(force: bool = False):
    """Build examples/main_cc from the reference's main.cc + CornellBox.cpp,
    and tests/cpp/scene_unchanged_check (the reference's CornellBox against
    rtp_cornell_box); None when the reference is absent (the GPU box)."""
    if not all(os.path.exists(os.path.join(REFERENCE_DIR, f)) for f in REFERENCE_SOURCES):
        return None
    lib = build()
    compat = os.path.join(ROOT, "include", "vtkm_compat")
    inc = os.path.join(ROOT, "include")
    hdrs = [os.path.join(inc, "rtp", f) for f in ("vtkm_compat.hpp", "rendering.hpp")] + [os.path.join(inc, "rtp.h")]
    cxx = [os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-I", compat, "-I", inc, "-iquote", REFERENCE_DIR]
    objdir = os.path.join(ROOT, "examples", "obj")
    os.makedirs(objdir, exist_ok=True)
    objs = {}
    for f in REFERENCE_SOURCES:
        src = os.path.join(REFERENCE_DIR, f)
        obj = os.path.join(objdir, f + ".o")
        if force or not os.path.exists(obj) or any(os.path.getmtime(d) > os.path.getmtime(obj) for d in hdrs + [src]):
            with open(src, "rb") as fh:
                res = subprocess.run(cxx + ["-x", "c++", "-", "-c", "-o", obj], stdin=fh, cwd=compat,
                                     capture_output=True, text=True)
            if res.returncode != 0:
                raise RuntimeError(f"g++ failed on the unchanged {f}:\n{res.stderr[-4000:]}")
        objs[f] = obj
    targets = {MAIN_UNCHANGED: [objs["main.cc"], objs["CornellBox.cpp"]],
               SCENE_CHECK: [os.path.join(ROOT, "tests", "cpp", "scene_unchanged_check.cpp"), objs["CornellBox.cpp"]]}
    for exe, ins in targets.items():
        deps = ins + hdrs + [lib]
        if force or not os.path.exists(exe) or any(os.path.getmtime(d) > os.path.getmtime(exe) for d in deps):
            rel = os.path.relpath(HERE, os.path.dirname(exe))
            res = subprocess.run(cxx + ins + ["-L", HERE, "-lrtp", f"-Wl,-rpath,$ORIGIN/{rel}", "-o", exe], cwd=compat,
                                 capture_output=True, text=True)
            if res.returncode != 0:
                raise RuntimeError(f"g++ link failed for {exe}:\n{res.stderr[-4000:]}")
    return MAIN_UNCHANGED


ASAN_DIR = os.path.join(ROOT, "tests", "cpp", "asan")
# programs linked against the host-sanitized library sources (not librtp.so)
ASAN_PROGRAMS = {
    os.path.join(ASAN_DIR, "asan_scene"): os.path.join(ROOT, "tests", "cpp", "asan_scene.cpp"),
    os.path.join(ASAN_DIR, "shim_check"): os.path.join(ROOT, "tests", "cpp", "shim_check.cpp"),
}
# AddressSanitizer + UBSan on host code only (GPU sanitizers are not available
# on the pool): each -fsanitize= directly after -Xarch_host.  The sanitizer
# runtime links statically into the executables (clang's default).
ASAN_HOST = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
             "-Xarch_host", "-fno-omit-frame-pointer", "-Xarch_host", "-fno-sanitize-recover=undefined"]


def build_asan(force: bool = False) -> list[str]:
    """Host-sanitized builds of the library's sources linked into the test
    drivers of tests/cpp (one object per source, cached by mtime)."""
    os.makedirs(ASAN_DIR, exist_ok=True)
    base = [hipcc(), "-O1", "-g", f"--offload-arch={ARCH}", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
            "-fno-slp-vectorize", *ASAN_HOST]
    hdrs = [os.path.join(CSRC, f) for f in HEADERS]
    newest_hdr = max(os.path.getmtime(h) for h in hdrs if os.path.exists(h))
    objs = []
    for s in SOURCES:
        src = os.path.join(CSRC, s)
        obj = os.path.join(ASAN_DIR, s + ".o")
        if force or not os.path.exists(obj) or os.path.getmtime(obj) < max(os.path.getmtime(src), newest_hdr):
            res = subprocess.run([*base, "-fPIC", "-c", src, "-o", obj + ".tmp"], capture_output=True, text=True)
            if res.returncode != 0:
                raise RuntimeError(f"hipcc (asan) failed for {s}:\n{res.stderr}")
            os.replace(obj + ".tmp", obj)
        objs.append(obj)
    inc = os.path.join(ROOT, "include")
    built = []
    for exe, src in ASAN_PROGRAMS.items():
        deps = objs + [src, os.path.join(inc, "rtp.h"), os.path.join(inc, "rtp", "rendering.hpp")]
        if force or not os.path.exists(exe) or any(os.path.getmtime(d) > os.path.getmtime(exe) for d in deps):
            # the driver is host C++ (g++-style, like build_cpp), the link
            # pulls in the HIP runtime and the static sanitizer runtimes
            res = subprocess.run([*base, "-x", "c++", "-I", inc, "-c", src, "-o", exe + ".o"], capture_output=True,
                                 text=True)
            if res.returncode == 0:
                res = subprocess.run([hipcc(), "-fsanitize=address,undefined", exe + ".o", *objs, "-o", exe],
                                     capture_output=True, text=True)
            if res.returncode != 0:
                raise RuntimeError(f"hipcc (asan) build failed for {src}:\n{res.stderr[-4000:]}")
        built.append(exe)
    return built


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
    print("\n".join(build_cpp(force="--force" in sys.argv)))
    print(build_main_unchanged(force="--force" in sys.argv))
