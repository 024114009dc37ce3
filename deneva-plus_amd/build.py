"""Builds libdvcc.so (HIP kernels for gfx950 + epoch runtime + host epoch
builder) in-tree at deneva-plus_amd/build/libdvcc.so.

    python deneva-plus_amd/build.py [--force]

Plain hipcc/g++ invocations (no cmake/ninja); objects are rebuilt when their
sources or headers are newer.
"""
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
# DVCC_BUILD_DIR / DVCC_DEFINES: experiment variants (tools/exp_pass.py) only
OUT = os.environ.get("DVCC_BUILD_DIR") or os.path.join(PKG, "build")
DEFINES = os.environ.get("DVCC_DEFINES", "").split()
LIB = os.path.join(OUT, "libdvcc.so")
INCLUDE = os.path.join(ROOT, "include")
ARCH = os.environ.get("DVCC_OFFLOAD_ARCH", "gfx950")

HEADERS = [os.path.join(INCLUDE, "dvcc.h"), os.path.join(CSRC, "dvcc_internal.h"),
           os.path.join(CSRC, "dvcc_common.h"), os.path.join(CSRC, "dvcc_tpcc.h")]
HIP_SRCS = ["dvcc_kernels.hip", "dvcc_rounds.hip", "dvcc_prefix.hip", "dvcc_carry.hip", "dvcc_comm.hip", "dvcc_tpcc.hip",
            "dvcc_runtime.hip"]
CPP_SRCS = ["ycsb_gen.cpp", "tpcc_gen.cpp", "wire.cpp"]


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)


def build(force=False, verbose_resources=False):
    os.makedirs(OUT, exist_ok=True)
    objs = []
    for s in HIP_SRCS:
        src = os.path.join(CSRC, s)
        obj = os.path.join(OUT, s.replace(".hip", ".o"))
        objs.append(obj)
        if force or _newer(obj, [src] + HEADERS):
            cmd = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
                   "-I", INCLUDE, "-I", CSRC, "-c", src, "-o", obj] + DEFINES
            if verbose_resources:
                cmd.insert(1, "-Rpass-analysis=kernel-resource-usage")
            _run(cmd)
    for s in CPP_SRCS:
        src = os.path.join(CSRC, s)
        obj = os.path.join(OUT, s.replace(".cpp", ".o"))
        objs.append(obj)
        if force or _newer(obj, [src] + HEADERS):
            _run(["g++", "-O2", "-std=c++17", "-fPIC", "-ffp-contract=off", "-I", INCLUDE,
                  "-c", src, "-o", obj])
    if force or _newer(LIB, objs):
        _run(["hipcc", f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB] + objs
             + ["-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"])
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose_resources="--resources" in sys.argv)
