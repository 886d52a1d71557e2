"""The oracle (oracle/rt_oracle.c) against fixtures generated from the reference
itself (tests/golden/make_golden.py). CPU only."""
import ctypes
import hashlib

import numpy as np
import pytest

from conftest import bits, golden, golden_npy, sha, unhex


def test_glibc_stream_matches_libc(oracle_mod):
    libc = ctypes.CDLL("libc.so.6")
    for seed in (1, 42, 2147483646):
        libc.srand(seed)
        want = np.array([libc.rand() for _ in range(2000)], dtype=np.int32)
        assert np.array_equal(oracle_mod.glibc_draws(seed, 2000), want)


def test_rng_kat(oracle_mod):
    rk = golden("rng_kat.json")
    for c in rk["glibc"]:
        assert oracle_mod.glibc_draws(c["seed"], len(c["draws"])).tolist() == c["draws"]
    for c in rk["counter"]:
        got = oracle_mod.counter_draws(int(c["seed"]), c["pixel"], c["sample"], len(c["draws"]))
        assert got.tolist() == c["draws"]


def test_reference_main_glibc_10spp(oracle_mod):
    """Reference main() semantics (serial glibc stream, seed 1): the P3 bytes
    equal the reference binary's (main.cc:51-92 at 10 spp)."""
    g = golden("reference_glibc.json")
    two = oracle_mod.scene_two_spheres()
    _, rgb, _ = oracle_mod.render(two, oracle_mod.camera_default(), 400, 225, 10,
                                  rng=oracle_mod.RNG_GLIBC, seed=1)
    assert hashlib.md5(oracle_mod.ppm_p3(rgb)).hexdigest() == g["glibc_two_400x225x10_p3_md5"]


@pytest.mark.slow
def test_reference_main_glibc_100spp(oracle_mod):
    g = golden("reference_glibc.json")
    _, rgb, _ = oracle_mod.render(oracle_mod.scene_two_spheres(), oracle_mod.camera_default(),
                                  400, 225, 100, rng=oracle_mod.RNG_GLIBC, seed=1)
    assert hashlib.md5(oracle_mod.ppm_p3(rgb)).hexdigest() == g["reference_main_p3_md5"]


def test_counter_two_sphere_cases(oracle_mod):
    fx = golden("counter_two.json")
    sph = np.array(unhex(fx["spheres"]))
    cam = np.array(unhex(fx["camera"]))
    assert np.array_equal(cam, oracle_mod.camera_default())
    assert np.array_equal(sph, oracle_mod.scene_two_spheres())
    for c in fx["cases"]:
        if c["width"] * c["height"] * c["spp"] > 400 * 225 * 10:
            continue  # 100 spp case: covered on the GPU and by make_golden
        acc, rgb, rays = oracle_mod.render(sph, cam, c["width"], c["height"], c["spp"],
                                           c["max_depth"], c["seed"], c["row_offset"],
                                           c["row_stride"], threads=8)
        assert sha(acc) == c["accum_sha256"], c
        assert hashlib.md5(oracle_mod.ppm_p3(rgb)).hexdigest() == c["p3_md5"]
        assert rays == c["rays"]
        if "accum_npy" in c:
            assert np.array_equal(bits(acc), bits(golden_npy(c["accum_npy"])))


def test_final_scene_and_camera(oracle_mod, final_scene):
    fx = golden("counter_final.json")
    assert fx["n"] == len(final_scene) == 485
    assert np.array_equal(final_scene, oracle_mod.scene_random_spheres(1))
    assert np.array_equal(np.array(unhex(fx["camera_1200x800"])),
                          oracle_mod.camera_look_at(aspect=1200 / 800))


def test_counter_final_small(oracle_mod, final_scene):
    fx = golden("counter_final.json")
    for c in fx["cases"]:
        cam = np.array(unhex(c["camera"]))
        acc, rgb, rays = oracle_mod.render(final_scene, cam, c["width"], c["height"], c["spp"],
                                           c["max_depth"], c["seed"], threads=8)
        assert sha(acc) == c["accum_sha256"]
        assert rays == c["rays"]


def test_sampled_pixels_full_size(oracle_mod, final_scene):
    """Pixels of C3 (1200x800x100) and C4 (3840x2160x500) at full spp."""
    fx = golden("counter_final.json")
    for grp in fx["sampled"]:
        cam = np.array(unhex(grp["camera"]))
        pix = grp["pixels"][:6]
        ii = [p["i"] for p in pix]
        jj = [grp["height"] - 1 - p["row"] for p in pix]
        out, _ = oracle_mod.render_pixels(final_scene, cam, grp["width"], grp["height"],
                                          grp["spp"], ii, jj, grp["max_depth"], grp["seed"])
        want = np.array([unhex(p["accum"]) for p in pix])
        assert np.array_equal(bits(out), bits(want))


def _kat_spheres(c, final_scene):
    return final_scene if c["spheres"] == "final" else np.array(unhex(c["spheres"]))


def test_world_hit_kat(oracle_mod, final_scene):
    cases = golden("kat_hit.json")
    for c in cases:
        sph = _kat_spheres(c, final_scene)
        idx, rec = oracle_mod.world_hit(sph, unhex(c["o"]), unhex(c["d"]), unhex(c["tmin"]),
                                        unhex(c["tmax"]))
        assert idx == c["expect_index"], c["name"]
        if idx >= 0:
            want = [float.fromhex(x) for x in c["expect"][:7]]
            got = rec[:7]
            for g, w in zip(got, want):
                assert (np.isnan(g) and np.isnan(w)) or bits(g) == bits(w), c["name"]
            assert int(rec[7]) == int(c["expect"][7])


def test_trace_kat_self_consistent(oracle_mod, final_scene):
    """Per-bounce path records (written by the oracle once it was shown
    bit-equal to the reference) replay identically."""
    two = oracle_mod.scene_two_spheres()
    for c in golden("trace_kat.json")[:8]:
        sph = two if c["scene"] == "two" else final_scene
        cam = (oracle_mod.camera_default() if c["scene"] == "two"
               else oracle_mod.camera_look_at(aspect=c["width"] / c["height"]))
        col, bounces = oracle_mod.trace_sample(sph, cam, c["width"], c["height"], c["i"], c["j"],
                                               c["s"])
        assert [x.hex() for x in col] == c["color"]
        assert len(bounces) == len(c["bounces"])
        for b, w in zip(bounces, c["bounces"]):
            assert b["index"] == w["index"] and b["draws_after"] == w["draws_after"]
            assert [x.hex() for x in b["o"]] == w["o"]


def test_reference_build_matches_fixture(oracle_mod):
    """When the reference build is present, it still produces the fixtures."""
    if not oracle_mod.have_ref():
        pytest.skip("oracle/_ref not built (reference absent)")
    fx = golden("counter_two.json")
    c = fx["cases"][0]
    out, st = oracle_mod.run_ref(["--scene", "two", "--width", str(c["width"]), "--height",
                                  str(c["height"]), "--spp", str(c["spp"])])
    assert hashlib.md5(out).hexdigest() == c["p3_md5"]
    assert st["rays"] == c["rays"]
