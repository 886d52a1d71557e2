"""psrt_trace's FP32 pre-decision of random_in_unit_sphere's test against the
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
