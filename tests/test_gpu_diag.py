"""The diagnostic kernel variant (tuning knob stamps = 1: psrt_trace<kStamps = true>,
DESIGN.md §4 section clocks, lane-utilisation probes and the wave timeline)
renders the same bits and rays as the product kernel and prints its
measurement lines. It is the only non-default variant the library builds
besides the counting one (RT_FLAG_CULL_STATS), so the GPU suite runs it."""
import json

import numpy as np
import pytest

import petershirleyraytracer_amd as P
from conftest import bits

pytestmark = pytest.mark.gpu


def test_stamps_variant_same_bits_and_reports(final_scene, knobs, capfd):
    cam = P.camera_look_at(aspect=96 / 64)
    a, ra, sa = P.render(final_scene, cam, 96, 64, 4)
    knobs("stamps", 1)
    b, rb, sb = P.render(final_scene, cam, 96, 64, 4)
    knobs("stamps", 0)
    assert np.array_equal(bits(a), bits(b)) and np.array_equal(ra, rb)
    assert (sa["rays"], sa["rays_traced"]) == (sb["rays"], sb["rays_traced"])
    err = capfd.readouterr().err
    lines = {k: json.loads(l)[k] for l in err.splitlines() if l.startswith("{")
             for k in json.loads(l)}
    assert {"psrt_util", "psrt_waves", "psrt_sections"} <= set(lines), err[-2000:]
    sec = lines["psrt_sections"]
    assert abs(sum(sec[k] for k in ("refill", "hit_quick", "scatter", "fill_shade", "traverse"))
               - 1.0) < 1e-6 + 0.5  # shares of the wave cycles (the hit_quick split is inside)
    assert sec["wave_trips"] > 0 and lines["psrt_waves"]["waves"] > 0
