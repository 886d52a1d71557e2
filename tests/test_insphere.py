"""Host checks of psrt_trace arithmetic shortcuts: the FP32 pre-decision of
random_in_unit_sphere's test against the
FP64 test, CPU (tests/host/insphere_check.c): every triple it decides gets
the FP64 answer, random and near-surface triples."""
import os
import subprocess

from conftest import ROOT


def test_fp32_in_sphere_predecision_matches_fp64(tmp_path):
    exe = str(tmp_path / "insphere_check")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-Wall", "-o", exe,
                    os.path.join(ROOT, "tests", "host", "insphere_check.c"), "-lm"], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    ok, decided, undecided = r.stdout.split()
    assert ok == "ok" and int(decided) > 18_000_000 and int(undecided) > 0


def test_pm1_one_add_conversion_exhaustive(tmp_path):
    """pm1_raw (psrt_device.h) as one FP64 add equals random_double(-1, 1)
    (random.h:10-14) of rand() = raw >> 1 for all 2^31 even raw draws."""
    exe = str(tmp_path / "pm1_check")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-Wall", "-o", exe,
                    os.path.join(ROOT, "tests", "host", "pm1_check.c")], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.split() == ["ok", str(1 << 31)]


def test_fp32_pre_reject_never_rejects_a_reference_hit(tmp_path):
    """test_sphere's FP32 pre-reject (psrt_kernels.hip Pre32) on 8.2 M
    adversarial origins 1e-13 .. 1e2 outside spheres (the r = 1000 ground
    included), bt around D / |d|, at scene scales 1 down to 2^-90: whenever
    it rejects, the reference's FP64 test (sphere.cc:6-31 over [0, bt])
    accepts no root. The same check with the margins removed finds
    violations, and so does the r04 floor of R (2^-100) at the tiny scales
    (ADVICE r04): the test has teeth."""
    src = os.path.join(ROOT, "tests", "host", "pre32_check.c")
    exe = str(tmp_path / "pre32_check")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-Wall", "-o", exe, src, "-lm"], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    ok, cases, rejected = r.stdout.split()
    assert ok == "ok" and int(cases) == 8_200_000 and int(rejected) > 1_000_000
    old = str(tmp_path / "pre32_old_floor")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-DR_FLOOR=0x1p-100", "-o", old, src, "-lm"],
                   check=True)
    r = subprocess.run([old], capture_output=True, text=True, timeout=120)
    assert r.returncode == 1 and "violations" in r.stdout
