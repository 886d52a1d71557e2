"""Register budgets read from the built library's gfx950 code object (no GPU).

psrt_reduce_lean and psrt_fold_stats must fit beside a resident psrt_trace
launch (frames in flight): measured on MI355X
(scripts/coresident_probe.py, profiles/r06_drain), a kernel with 16 SGPRs
starts beside the trace and one with 20 does not, while 29 VGPRs still fit;
LDS is all but ~10 KB taken. The trace's own counts set that room, so they
are pinned too: a change that grows them has to be measured again."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "petershirleyraytracer_amd", "lib", "libpsrt.so")
LLVM = "/opt/rocm/lib/llvm/bin"


def _kernels(tmp_path):
    bundler = os.path.join(LLVM, "clang-offload-bundler")
    readelf = os.path.join(LLVM, "llvm-readelf")
    if not (os.path.exists(LIB) and shutil.which("objcopy") and os.path.exists(bundler)
            and os.path.exists(readelf)):
        pytest.skip("library or LLVM tools absent")
    fb, co = tmp_path / "fb.bin", tmp_path / "k.co"
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", LIB, str(fb)],
                   check=True)
    subprocess.run([bundler, "--unbundle", "--type=o",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fb}",
                    f"--output={co}"], check=True)
    notes = subprocess.run([readelf, "--notes", str(co)], check=True, capture_output=True,
                           text=True).stdout
    # the metadata lists one map per kernel: collect its keys up to the next "- "
    out, cur = {}, {}
    for line in notes.splitlines():
        m = re.match(r"\s*(-\s+)?\.(\w+):\s+(\S+)", line)
        if not m:
            continue
        if m.group(1) and cur:
            if "name" in cur:
                out[cur["name"]] = cur
            cur = {}
        cur[m.group(2)] = m.group(3)
    if "name" in cur:
        out[cur["name"]] = cur
    return out


def _find(ks, part):
    hits = [v for k, v in ks.items() if part in k]
    assert hits, part
    return hits


def test_lean_kernels_fit_beside_the_trace(tmp_path):
    ks = _kernels(tmp_path)
    for name in ("psrt_reduce_lean", "psrt_fold_stats"):
        for k in _find(ks, name):
            assert int(k["sgpr_count"]) <= 16, (name, k["sgpr_count"])
            assert int(k["vgpr_count"]) <= 32, (name, k["vgpr_count"])
            assert int(k["group_segment_fixed_size"]) == 0, name
            assert int(k["private_segment_fixed_size"]) == 0, name


def test_trace_register_counts_pinned(tmp_path):
    """The product trace variant (BVH, LDS scene, not the counting one)."""
    ks = _kernels(tmp_path)
    (k,) = _find(ks, "psrt_traceILb1ELb0ELb1ELb0E")
    assert int(k["vgpr_count"]) == 80 and int(k["sgpr_count"]) <= 112, k
