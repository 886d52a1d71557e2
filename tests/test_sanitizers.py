"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer.

The product's host C++ that takes caller input or builds the culling
structures (psrt_scenefile.cpp: the scene-file parser; psrt_bvh.cpp: BVH,
grid, block and neighbour lists; psrt_scene.cpp: scenes, cameras,
write_color) and the oracle's C restatement, built with
-fsanitize=address,undefined -fno-sanitize-recover=all and run over the
committed scene files, random scenes, a mutation fuzz of rt_scene_parse and
the culling invariants of tests/host/bvh_check.cc. Any sanitizer report
aborts the program, so a clean exit is the pass. CPU only (no HIP code).
"""
import os
import subprocess

import pytest

from conftest import ROOT

CSRC = os.path.join(ROOT, "petershirleyraytracer_amd", "csrc")
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer",
       "-g", "-O1"]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


def _run(exe, *args, timeout=300):
    r = subprocess.run([exe, *args], capture_output=True, text=True, timeout=timeout, env=ENV)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    return r.stdout


def test_scenefile_parser_and_culling_build_fuzzed_under_sanitizers(tmp_path):
    exe = str(tmp_path / "scenefile_fuzz")
    subprocess.run(["g++", *SAN, "-std=c++17", "-Wall", "-ffp-contract=off",
                    f"-I{os.path.join(ROOT, 'include')}", "-o", exe,
                    os.path.join(ROOT, "tests", "host", "scenefile_fuzz.cc"),
                    os.path.join(CSRC, "psrt_scenefile.cpp"), os.path.join(CSRC, "psrt_scene.cpp"),
                    os.path.join(CSRC, "psrt_bvh.cpp")], check=True)
    scenes = [os.path.join(ROOT, "scenes", f) for f in sorted(os.listdir(os.path.join(ROOT, "scenes")))]
    out = _run(exe, *scenes)
    last = out.strip().splitlines()[-1].split()
    assert last[0] == "ok" and not any(l.startswith("FAIL") for l in out.splitlines()), out[-2000:]
    assert int(last[1]) > 100 and int(last[2]) > 100  # the fuzz reached both outcomes


def test_culling_invariants_under_sanitizers(tmp_path):
    exe = str(tmp_path / "bvh_check_san")
    subprocess.run(["g++", *SAN, "-std=c++17", "-Wall", f"-I{os.path.join(ROOT, 'include')}",
                    "-o", exe, os.path.join(ROOT, "tests", "host", "bvh_check.cc"),
                    os.path.join(CSRC, "psrt_bvh.cpp"), os.path.join(CSRC, "psrt_scene.cpp")],
                   check=True)
    out = _run(exe, timeout=600)
    assert not any(l.startswith("FAIL") for l in out.splitlines()), out


def test_oracle_restatement_under_sanitizers(tmp_path):
    exe = str(tmp_path / "oracle_san")
    subprocess.run(["gcc", *SAN, "-std=c99", "-Wall", "-Wno-unused-function", "-ffp-contract=off",
                    "-pthread", "-o", exe, os.path.join(ROOT, "tests", "host", "oracle_san.c"),
                    os.path.join(ROOT, "oracle", "rt_oracle.c"),
                    os.path.join(ROOT, "oracle", "rt_oracle_mat.c"), "-lm"], check=True)
    assert _run(exe).strip() == "ok"
