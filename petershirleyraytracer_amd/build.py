"""Build the native pieces in-tree (they travel to the GPU box with the repo).

  lib/libpsrt.so      HIP kernels + C ABI (include/rt.h), gfx950, -ffp-contract=off
  bin/raytracer       the C++ host (reference main() drop-in) over the C ABI

hipcc cross-compiles for gfx950 without a GPU, so this runs in the CPU container.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB_DIR = os.path.join(PKG, "lib")
BIN_DIR = os.path.join(PKG, "bin")
LIB = os.path.join(LIB_DIR, "libpsrt.so")
HOST_BIN = os.path.join(BIN_DIR, "raytracer")

ARCH = os.environ.get("PSRT_ARCH", "gfx950")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"

# -ffp-contract=off is load-bearing: bitwise parity with the reference needs
# every x*y+z to stay a separate multiply and add.
COMMON = ["-O3", "-ffp-contract=off", "-std=c++17", "-Wall"]

LIB_SOURCES = ["psrt_kernels.hip", "psrt_mat.hip", "psrt_capi.hip", "psrt_group.cpp", "psrt_scene.cpp",
               "psrt_scenefile.cpp", "psrt_bvh.cpp"]
HOST_SOURCES = [os.path.join("host", "raytracer_main.cc")]


def _newer(target: str, sources) -> bool:
    if not os.path.exists(target):
        return False
    t = os.path.getmtime(target)
    return all(os.path.getmtime(s) <= t for s in sources)


def _deps():
    out = []
    for d in (CSRC, os.path.join(ROOT, "include")):
        for dp, _, fs in os.walk(d):
            out.extend(os.path.join(dp, f) for f in fs
                       if f.endswith((".h", ".hpp", ".hip", ".cpp", ".cc")))
    return out


def build_lib(force: bool = False, verbose: bool = False, out: str = LIB,
              defines=()) -> str:
    os.makedirs(LIB_DIR, exist_ok=True)
    srcs = [os.path.join(CSRC, s) for s in LIB_SOURCES]
    if not force and _newer(out, _deps()):
        return out
    extra = os.environ.get("PSRT_HIPCC_FLAGS", "").split()  # tuning builds only
    cmd = [HIPCC, f"--offload-arch={ARCH}", *COMMON, *extra, *[f"-D{d}" for d in defines],
           "-fPIC", "-shared", "-o", out, *srcs]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=CSRC)
    return out


def build_host(force: bool = False, verbose: bool = False) -> str:
    """The C++ host app links libpsrt.so (rpath $ORIGIN/../lib)."""
    os.makedirs(BIN_DIR, exist_ok=True)
    srcs = [os.path.join(CSRC, s) for s in HOST_SOURCES]
    if not all(os.path.exists(s) for s in srcs):
        return ""
    if not force and _newer(HOST_BIN, _deps() + [LIB]):
        return HOST_BIN
    cmd = ["g++", "-O2", "-ffp-contract=off", "-std=c++17", "-Wall",
           f"-I{os.path.join(ROOT, 'include')}", "-o", HOST_BIN, *srcs,
           f"-L{LIB_DIR}", "-lpsrt", "-Wl,-rpath,$ORIGIN/../lib"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=CSRC)
    return HOST_BIN


def build_all(force: bool = False, verbose: bool = False) -> None:
    build_lib(force, verbose)
    build_host(force, verbose)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv, verbose=True)
