"""psrt_trace's camera-ray division (div_by: RN(1/d) and two FMA corrections)
against IEEE division, CPU (tests/host/div_by_check.c)."""
import os
import subprocess

from conftest import ROOT


def test_div_by_matches_ieee_division(tmp_path):
    exe = str(tmp_path / "div_by_check")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-Wall", "-o", exe,
                    os.path.join(ROOT, "tests", "host", "div_by_check.c"), "-lm"], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok "), r.stdout
    assert int(r.stdout.split()[1]) > 3_000_000
