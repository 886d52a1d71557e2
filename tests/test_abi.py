"""The C-ABI boundary (include/rt.h) without a GPU: the library loads, exports
every declared symbol, its host helpers agree with the oracle and the
reference fixtures, and render calls fail loudly (no CPU fallback)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from conftest import ROOT, golden, have_gpu, unhex

import petershirleyraytracer_amd as P
from petershirleyraytracer_amd import _lib
from petershirleyraytracer_amd.build import LIB


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "rt.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rt_[a-z0-9_]+)\s*\(", src)))


def test_library_built():
    assert os.path.exists(LIB), "run __graft_entry__.build() first"


def test_exports_every_declared_symbol():
    L = C.CDLL(LIB)
    decl = declared_symbols()
    assert len(decl) >= 19
    for name in decl:
        assert hasattr(L, name), name
    assert sorted(_lib.EXPORTS) == decl


def test_abi_version_and_info():
    L = _lib.load()
    hdr = open(os.path.join(ROOT, "include", "rt.h")).read()
    want = int(re.search(r"#define RT_ABI_VERSION (\d+)", hdr).group(1))
    assert L.rt_abi_version() == want == _lib.ABI_VERSION == 7
    assert b"gfx950" in L.rt_build_info()


def test_rows_owned():
    assert P.rows_owned(800, 0, 1) == 800
    assert P.rows_owned(800, 3, 8) == 100
    assert P.rows_owned(801, 0, 8) == 101
    assert P.rows_owned(5, 4, 8) == 1
    assert P.rows_owned(5, 5, 8) == 0
    assert P.rows_owned(5, 0, 0) == 0
    for h in (1, 7, 225, 800):
        for w in (1, 2, 3, 8):
            assert sum(P.rows_owned(h, r, w) for r in range(w)) == h


def test_cameras_match_reference_fixtures(oracle_mod):
    two = golden("counter_two.json")
    assert np.array_equal(P.camera_default(), np.array(unhex(two["camera"])))
    fin = golden("counter_final.json")
    assert np.array_equal(P.camera_look_at(aspect=1200 / 800),
                          np.array(unhex(fin["camera_1200x800"])))
    for c in fin["cases"]:
        assert np.array_equal(P.camera_look_at(aspect=c["width"] / c["height"]),
                              np.array(unhex(c["camera"])))
    for aspect in (1.0, 16 / 9, 3840 / 2160, 0.5):
        assert np.array_equal(P.camera_look_at(aspect=aspect),
                              oracle_mod.camera_look_at(aspect=aspect))


def test_scenes_match_reference(final_scene):
    assert np.array_equal(P.scene_two_spheres(), np.array(unhex(golden("counter_two.json")["spheres"])))
    assert np.array_equal(P.scene_random_spheres(1), final_scene)


def test_scene_generator_tracks_glibc(oracle_mod):
    for seed in (2, 99, 123456):
        assert np.array_equal(P.scene_random_spheres(seed), oracle_mod.scene_random_spheres(seed))


def test_host_quantize_matches_oracle(oracle_mod):
    rng = np.random.default_rng(0)
    acc = rng.uniform(0, 120, size=(17, 23, 3))
    acc[0, 0] = [0.0, 100.0, 1e-30]
    acc[1, 1] = [99.8001, 99.9, 1e9]
    for spp in (1, 10, 100):
        assert np.array_equal(P.quantize(acc, spp), oracle_mod.quantize(acc, spp))


def test_ppm_p3_format(oracle_mod):
    rgb = np.arange(2 * 3 * 3, dtype=np.uint8).reshape(2, 3, 3)
    assert P.ppm_p3(rgb) == oracle_mod.ppm_p3(rgb)
    assert P.ppm_p3(rgb).startswith(b"P3\n3 2\n255\n0 1 2\n")


def test_bad_arguments_are_errors():
    L = _lib.load()
    cam = _lib.RtCamera()
    p = P.params(1, 1, 1)
    acc = (C.c_double * 3)()
    assert L.rt_render(None, 0, C.byref(cam), C.byref(p), acc, None, None) == -1
    assert b"width/height" in L.rt_last_error()
    p = P.params(4, 4, 0)
    assert L.rt_render(None, 0, C.byref(cam), C.byref(p), acc, None, None) == -1
    p = P.params(4, 4, 1, row_offset=-1)
    assert L.rt_render(None, 0, C.byref(cam), C.byref(p), acc, None, None) == -1
    p = P.params(4, 4, 1, row_stride=0)
    assert L.rt_render(None, 0, C.byref(cam), C.byref(p), acc, None, None) == -1
    # row_offset >= height: a shard that owns no rows (more ranks than rows)
    # is valid and may pass no output buffers; it fails only for want of a device
    p = P.params(4, 4, 1, row_offset=4)
    assert L.rt_rows_owned(4, 4, 1) == 0
    assert L.rt_render(None, 0, C.byref(cam), C.byref(p), None, None, None) in (
        (0,) if have_gpu() else (-2, -3))
    assert L.rt_render(None, 0, None, C.byref(p), acc, None, None) == -1


def test_group_bad_arguments_are_errors():
    """rt_group_* argument checks need no device; without one, creating a
    group fails with the context's error and leaves no group behind."""
    L = _lib.load()
    out = C.c_void_p()
    devs = (C.c_int * 2)(0, 0)
    assert L.rt_group_create(None, 2, C.byref(out)) == -1
    assert L.rt_group_create(devs, 0, C.byref(out)) == -1
    assert L.rt_group_create(devs, 2, None) == -1
    assert L.rt_group_size(None) == 0 and not L.rt_group_context(None, 0)
    assert L.rt_group_destroy(None) == 0
    p = P.params(4, 4, 1)
    assert L.rt_group_render(None, C.byref(p), None, None, None) == -1
    assert L.rt_group_set_scene(None, None, 0, None) == -1
    if not have_gpu():
        rc = L.rt_group_create(devs, 2, C.byref(out))
        assert rc in (-2, -3) and not out.value, rc


@pytest.mark.skipif(have_gpu(), reason="checks the no-device path")
def test_render_without_device_fails_loudly():
    with pytest.raises(_lib.RtError) as e:
        P.render(P.scene_two_spheres(), P.camera_default(), 8, 4, 1)
    assert "RT_E_NODEVICE" in str(e.value) or "RT_E_HIP" in str(e.value)
    with pytest.raises(_lib.RtError):
        P.Context(0)


def test_product_does_not_import_oracle():
    """The product package must not reach the checker."""
    pkg = os.path.join(ROOT, "petershirleyraytracer_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith((".py", ".cpp", ".hip", ".h", ".cc")):
                txt = open(os.path.join(dp, f)).read()
                assert "import oracle" not in txt and "liboracle" not in txt, f
                assert "oracle/" not in txt, f


def test_tuning_knobs_without_device():
    """rt_context_set_tuning / get_tuning on the process defaults (ctx NULL)
    need no device: round trip, unknown names and non-finite values fail."""
    old = P.get_tuning("queue_k")
    assert old == 2.0 and P.get_tuning("sample_buf_mb") == 49152.0
    with P.tuning(queue_k=3.5, no_camlist=1):
        assert P.get_tuning("queue_k") == 3.5 and P.get_tuning("no_camlist") == 1.0
    assert P.get_tuning("queue_k") == old and P.get_tuning("no_camlist") == 0.0
    with pytest.raises(_lib.RtError, match="unknown knob"):
        P.set_tuning("no_such_knob", 1)
    with pytest.raises(_lib.RtError, match="finite"):
        P.set_tuning("queue_k", float("nan"))
    # every knob has a range: values whose integer casts would wrap are errors
    # and leave the old value in place
    for name, bad in (("sample_buf_mb", 1e20), ("sample_buf_mb", 0.5), ("queue_k", -1),
                      ("blocks_per_cu", -2), ("mat_batch", 1e12), ("flush_at", -5),
                      ("flush_at", 2.0 ** 40), ("linear_chunk", -1), ("no_lds", 2),
                      ("big_ratio", -1)):
        before = P.get_tuning(name)
        with pytest.raises(_lib.RtError, match="outside"):
            P.set_tuning(name, bad)
        assert P.get_tuning(name) == before, name


def test_render_path_reads_no_environment():
    """The library's knobs go through rt_context_set_tuning: no getenv in the
    product sources except RT_DEVICE (the one-shot entries' device, read once,
    include/rt.h)."""
    csrc = os.path.join(ROOT, "petershirleyraytracer_amd", "csrc")
    for dp, _, fs in os.walk(csrc):
        for f in fs:
            if not f.endswith((".hip", ".cpp", ".h", ".cc")):
                continue
            for m in re.finditer(r"getenv\(([^)]*)\)", open(os.path.join(dp, f)).read()):
                assert m.group(1) == '"RT_DEVICE"', (f, m.group(0))


def test_census_hooks_are_out_of_the_product_kernels():
    """The census's section duplicates live in psrt_ablate.h, included only by
    measurement builds (PSRT_ABLATE / PSRT_MAT_ABLATE non-zero)."""
    csrc = os.path.join(ROOT, "petershirleyraytracer_amd", "csrc")
    for f in ("psrt_kernels.hip", "psrt_mat.hip"):
        txt = open(os.path.join(csrc, f)).read()
        assert re.search(r"#if PSRT_(MAT_)?ABLATE ==", txt) is None, f
        assert "ablate_sink" not in txt, f


def test_out_arrays_are_checked():
    """render(out=...) rejects arrays of the wrong shape, type or layout before
    any device work."""
    sp, cam = P.scene_two_spheres(), P.camera_default()
    with pytest.raises(ValueError, match="accum"):
        P.render(sp, cam, 8, 4, 1, out=(np.zeros((4, 8, 2)), None))
    with pytest.raises(ValueError, match="accum"):
        P.render(sp, cam, 8, 4, 1, out=(np.zeros((4, 8, 3), np.float32), None))
    with pytest.raises(ValueError, match="rgb8"):
        P.render(sp, cam, 8, 4, 1, out=(np.zeros((4, 8, 3)), np.zeros((4, 8, 3))))
    with pytest.raises(ValueError, match="accum"):
        P.render(sp, cam, 8, 4, 1, out=(np.zeros((4, 8, 6))[:, :, ::2], None))


@pytest.mark.skipif(have_gpu(), reason="checks the no-device path")
def test_host_alloc_without_device_fails_loudly():
    with pytest.raises(_lib.RtError):
        P.host_array((4, 8, 3))
