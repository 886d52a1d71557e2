"""The roofline of a committed bench line is reproducible from the line itself
(VERDICT r04 item 1): achieved = (each kind of executed test x its issue
weight + traced rays x the shading ops) / the kernel's time per frame, with
bench.py's weights. CPU only: reads profiles/r05_final."""
import json
import os

import pytest

from conftest import ROOT

LINE = os.path.join(ROOT, "profiles", "r05_final", "bench_default.log")


def _line():
    with open(LINE) as f:
        return json.loads([ln for ln in f if ln.startswith("{")][-1])


@pytest.mark.skipif(not os.path.exists(LINE), reason="no committed r05 bench line")
def test_roofline_recomputes_from_the_line():
    import bench
    d = _line()
    r = d["roofline"]
    w = r["issue_weights_fp64_slots"]
    for k, v in bench.WEIGHTS.items():
        assert abs(w[k] - v) < 1e-3, k
    slots = (r["full_sphere_tests_per_launch"] * w["full_sphere_test"]
             + r["prerejects_per_launch"] * w["prereject"]
             + r["box_tests_evaluated_per_launch"] * w["box_test"]
             + r["root_box_tests_per_launch"] * w["root_box_test"]
             + r["rays_traced_per_launch"] * r["shade_ops_per_traced_ray"])
    achieved = slots / (r["avg_launch_ms"] * 1e-3) / 1e12
    assert abs(achieved - r["achieved"]) < 2e-3 * r["achieved"], (achieved, r["achieved"])
    assert abs(achieved / r["peak"] - r["frac"]) < 1e-3
    # the peak: 256 CUs x 4 SIMDs x 16 lanes x 2.4 GHz FP64 slots
    assert abs(r["peak"] - 256 * 64 * 2.4e9 / 1e12) < 0.01
    # the timed frame is bit-identical to the reference's pixels
    assert d["parity_vs_cpu"]["fp64_bit_identical"] is True
    assert d["cpu_baseline"]["kind"] == "reference"
