"""The C++ host side: the reference API surface (include/psrt/rtweekend.hpp,
include/raytracer/*.h) and the drop-in render (include/psrt/render.hpp)."""
import hashlib
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, golden, have_gpu

INC = os.path.join(ROOT, "include")
LIBDIR = os.path.join(ROOT, "petershirleyraytracer_amd", "lib")
REF_MAIN = "/root/reference/programs/main.cc"


def _compile(src, out, extra=()):
    cmd = ["g++", "-O2", "-ffp-contract=off", "-std=c++17", "-w", f"-I{INC}", "-o", out, src,
           f"-L{LIBDIR}", "-lpsrt", f"-Wl,-rpath,{LIBDIR}", *extra]
    subprocess.run(cmd, check=True)


def test_host_api_hit_kat(tmp_path, final_scene):
    exe = str(tmp_path / "kat")
    _compile(os.path.join(ROOT, "tests", "host", "kat_runner.cc"), exe)
    cases = golden("kat_hit.json")
    lines = []
    for c in cases:
        sph = final_scene.tolist() if c["spheres"] == "final" else \
            [[float.fromhex(v) for v in s] for s in c["spheres"]]
        toks = [str(len(sph))] + [float(v).hex() for s in sph for v in s] + c["o"] + c["d"] + \
            [c["tmin"], c["tmax"]]
        lines.append(" ".join(toks))
    p = tmp_path / "k.txt"
    p.write_text("\n".join(lines) + "\n")
    out = subprocess.run([exe, str(p)], check=True, capture_output=True).stdout.decode()
    res = out.strip().split("\n")
    for c, line in zip(cases, res):
        toks = line.split()
        assert int(toks[0]) == c["expect_index"], c["name"]
        if c["expect_index"] >= 0:
            assert toks[1:] == c["expect"], c["name"]
    assert res[len(cases)] == "flat 4 0,0,0,1 1,2,3,4 5,6,7,8 9,9,9,2"
    assert res[len(cases) + 1] == "bad rejected"


@pytest.mark.skipif(not os.path.exists(REF_MAIN), reason="reference sources absent")
def test_reference_main_compiles_against_our_api(tmp_path):
    """The reference's own main.cc, compiled against include/raytracer/ instead
    of its own headers, prints the reference's image byte for byte (main()
    unchanged: 400x225, 100 spp, glibc rand)."""
    exe = str(tmp_path / "refmain")
    # fed on stdin so that "sphere.h" etc. resolve to include/raytracer/, not to
    # the reference's own headers beside main.cc
    with open(REF_MAIN, "rb") as src:
        subprocess.run(["g++", "-O2", "-w", f"-I{os.path.join(INC, 'raytracer')}", "-x", "c++",
                        "-o", exe, "-"], stdin=src, check=True, cwd=str(tmp_path))
    out = subprocess.run([exe], check=True, capture_output=True, timeout=300).stdout
    assert hashlib.md5(out).hexdigest() == golden("reference_glibc.json")["reference_main_p3_md5"]


def test_host_app_built():
    exe = os.path.join(ROOT, "petershirleyraytracer_amd", "bin", "raytracer")
    assert os.path.exists(exe)
    if not have_gpu():
        r = subprocess.run([exe, "--width", "8", "--spp", "1"], capture_output=True)
        assert r.returncode == 1 and b"no HIP device" in r.stderr


@pytest.mark.gpu
def test_host_app_matches_reference_fixture(tmp_path):
    exe = os.path.join(ROOT, "petershirleyraytracer_amd", "bin", "raytracer")
    fx = golden("counter_two.json")
    c = fx["cases"][1]  # 400x225, 10 spp, depth 50, seed 0
    r = subprocess.run([exe, "--width", "400", "--spp", "10"], check=True, capture_output=True,
                       timeout=120)
    assert hashlib.md5(r.stdout).hexdigest() == c["p3_md5"]
    fin = golden("counter_final.json")["cases"][1]  # final 120x80x8
    out = tmp_path / "f.ppm"
    acc = tmp_path / "a.bin"
    subprocess.run([exe, "--scene", "final", "--width", "120", "--height", "80", "--spp", "8",
                    "-o", str(out), "--accum", str(acc)], check=True, timeout=120)
    assert hashlib.md5(out.read_bytes()).hexdigest() == fin["p3_md5"]
    a = np.fromfile(acc, dtype=np.float64)
    assert hashlib.sha256(a.tobytes()).hexdigest() == fin["accum_sha256"]


def test_host_app_rejects_bad_options(tmp_path):
    """bin/raytracer: malformed or out-of-range numbers, shards and device lists, and the book
    scene with --devices (materials render on one context), are usage errors
    (exit 2) before any device is touched, on any machine."""
    exe = os.path.join(ROOT, "petershirleyraytracer_amd", "bin", "raytracer")
    out = str(tmp_path / "x.ppm")
    for bad in (["--width", "8x"], ["--devices", "0,x"], ["--devices", "0,,1"], ["--devices", "-1"],
                ["--devices", "0"], ["--devices", "abc"], ["--scene", "book", "--devices", "2"],
                ["--rows", "1:2x"], ["--rows", "1"], ["--seed", "-3"], ["--seed", " -1"],
                ["--seed", "+4"], ["--aperture", "0.1q"],
                ["--width", "99999999999"], ["--seed", "99999999999999999999999"],
                ["--focus", "1e999"]):
        r = subprocess.run([exe, *bad, "-o", out, "--width", "8", "--height", "4", "--spp", "1"],
                           capture_output=True, text=True, timeout=60)
        assert r.returncode == 2, (bad, r.returncode, r.stderr)


@pytest.mark.gpu
def test_pinned_frames_bit_identical(tmp_path):
    """psrt::pinned_frame (rt_host_alloc memory, written by the device with no
    copy) holds the same bits as the ordinary frame through rt_render, a 1:3
    shard and a three-member device group, and is reused without reallocation
    (tests/host/pinned_frame.cc)."""
    exe = str(tmp_path / "pinned")
    _compile(os.path.join(ROOT, "tests", "host", "pinned_frame.cc"), exe)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", (r.stdout, r.stderr)
