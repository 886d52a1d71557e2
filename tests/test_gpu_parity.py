"""Parity of the HIP path (through the C ABI) with the reference, on an MI355X.

Expected values come from tests/golden/ (generated from the reference's own
sources) and, for anything not in a fixture, from the oracle restatement —
which tests/test_oracle.py pins to the same fixtures. The bar is bit-exact
FP64 accumulators and identical PPM bytes.
"""
import hashlib
import os

import numpy as np
import pytest

from conftest import GOLDEN, ROOT, bits, golden, golden_npy, sha, unhex

import petershirleyraytracer_amd as P
from petershirleyraytracer_amd.render import world_hit

pytestmark = pytest.mark.gpu


def test_device_visible():
    assert P.device_count() >= 1


# ---- numerics primitives ------------------------------------------------------

def _f64_inputs(n=1 << 16, seed=0):
    rng = np.random.default_rng(seed)
    x = np.concatenate([
        rng.uniform(0, 1, n), rng.uniform(0, 1e6, n), np.exp(rng.uniform(-700, 700, n)),
        rng.uniform(0, 1e-300, n // 4), np.array([0.0, -0.0, 1.0, 4.0, 2.0, 1e-320, 5e-324,
                                                  np.inf, np.nan, 1.7976931348623157e308]),
    ])
    y = np.concatenate([rng.uniform(1e-3, 10, len(x) - 10), np.array(
        [1.0, 3.0, -7.0, 0.1, 1e-310, 3.0, 2.0, 0.0, 1.0, 0.5])])
    return x, y


def _same(a, b):
    return np.all((bits(a) == bits(b)) | (np.isnan(a) & np.isnan(b)))


def test_sqrt_is_correctly_rounded():
    x, _ = _f64_inputs()
    assert _same(P.probe_f64(0, x), np.sqrt(x))


def test_kernel_sqrt_is_correctly_rounded():
    """sqrt_f64: the expansion's steps without its range handling, plus the
    full expansion behind a branch for 0, tiny, inf and NaN inputs."""
    x, _ = _f64_inputs(seed=2)
    rng = np.random.default_rng(8)
    edge = np.array([2.0**-767, np.nextafter(2.0**-767, 0), np.nextafter(2.0**-767, 1), 2.0**-1022,
                     5e-324, 1.7976931348623157e308, np.inf, -0.0, 0.0, -1.0, np.nan, 1e-300])
    x = np.concatenate([x, edge, np.abs(rng.normal(size=200000)) * 10.0 ** rng.integers(-320, 308, 200000)])
    got = P.probe_f64(6, x)
    with np.errstate(invalid="ignore"):
        assert _same(got, np.sqrt(x))
    # the same lanes mixed in one wave: fast and slow lanes side by side
    mix = np.where(np.arange(len(x)) % 3 == 0, 0.0, x)
    with np.errstate(invalid="ignore"):
        assert _same(P.probe_f64(6, mix), np.sqrt(mix))


def test_division_is_correctly_rounded():
    x, y = _f64_inputs(seed=1)
    assert _same(P.probe_f64(1, x, y), x / y)
    sx = np.random.default_rng(3).normal(size=200000)
    sy = np.random.default_rng(4).normal(size=200000)
    assert _same(P.probe_f64(1, sx, sy), sx / sy)


def test_no_fma_contraction():
    rng = np.random.default_rng(5)
    x = rng.normal(size=100000)
    y = rng.normal(size=100000)
    assert _same(P.probe_f64(4, x, y), x * y + x)
    assert _same(P.probe_f64(2, x, y), x * y)
    assert _same(P.probe_f64(3, x, y), x + y)


def test_ldexp_exact():
    x = np.random.default_rng(6).uniform(0.5, 1.0, 10000)
    k = -np.random.default_rng(7).integers(0, 60, 10000).astype(np.float64)
    assert _same(P.probe_f64(5, x, k), np.ldexp(x, k.astype(np.int64)))


# ---- sphere::hit / hittable_list::hit known answers ---------------------------

def test_world_hit_kat(final_scene):
    cases = golden("kat_hit.json")
    for c in cases:
        sph = final_scene if c["spheres"] == "final" else np.array(unhex(c["spheres"]))
        ray = np.array(unhex(c["o"]) + unhex(c["d"]) + [unhex(c["tmin"]), unhex(c["tmax"])])
        out = world_hit(sph, ray[None, :])[0]
        assert int(out[0]) == c["expect_index"], c["name"]
        if c["expect_index"] >= 0:
            want = np.array([float.fromhex(x) for x in c["expect"][:7]])
            got = out[1:8]
            assert _same(got, want), (c["name"], got, want)
            assert int(out[8]) == int(c["expect"][7]), c["name"]


# ---- whole renders vs reference fixtures -----------------------------------------

def test_counter_two_sphere_fixtures():
    fx = golden("counter_two.json")
    sph = np.array(unhex(fx["spheres"]))
    cam = np.array(unhex(fx["camera"]))
    for c in fx["cases"]:
        acc, rgb, st = P.render(sph, cam, c["width"], c["height"], c["spp"], c["max_depth"],
                                c["seed"], c["row_offset"], c["row_stride"])
        if "accum_npy" in c:
            want = golden_npy(c["accum_npy"])
            bad = np.argwhere(bits(acc) != bits(want))
            assert len(bad) == 0, (c, bad[:5], acc.reshape(-1)[:3], want.reshape(-1)[:3])
        assert sha(acc) == c["accum_sha256"], c
        assert hashlib.md5(P.ppm_p3(rgb)).hexdigest() == c["p3_md5"], c
        assert st["rays"] == c["rays"], c
        assert st["samples"] == acc.shape[0] * acc.shape[1] * c["spp"]
        assert 0 < st["kernel_ms"] <= st["total_ms"], st


def test_counter_final_fixtures(final_scene):
    fx = golden("counter_final.json")
    for c in fx["cases"]:
        cam = np.array(unhex(c["camera"]))
        acc, rgb, st = P.render(final_scene, cam, c["width"], c["height"], c["spp"],
                                c["max_depth"], c["seed"])
        if "accum_npy" in c:
            assert np.array_equal(bits(acc), bits(golden_npy(c["accum_npy"])))
        assert sha(acc) == c["accum_sha256"]
        assert hashlib.md5(P.ppm_p3(rgb)).hexdigest() == c["p3_md5"]
        assert st["rays"] == c["rays"]


def test_sampled_pixels_c3_c4(final_scene):
    """C3 (1200x800x100) in full, and C4 (3840x2160x500) one row per sampled
    pixel, against pixels the reference rendered."""
    fx = golden("counter_final.json")
    for grp in fx["sampled"]:
        w, h, spp = grp["width"], grp["height"], grp["spp"]
        cam = np.array(unhex(grp["camera"]))
        if w * h <= 1200 * 800:
            acc, _, _ = P.render(final_scene, cam, w, h, spp, grp["max_depth"], grp["seed"])
            for p in grp["pixels"]:
                assert np.array_equal(bits(acc[p["row"], p["i"]]), bits(unhex(p["accum"]))), p
        else:
            for p in grp["pixels"][:3]:
                acc, _, _ = P.render(final_scene, cam, w, h, spp, grp["max_depth"], grp["seed"],
                                     row_offset=p["row"], row_stride=h)
                assert acc.shape == (1, w, 3)
                assert np.array_equal(bits(acc[0, p["i"]]), bits(unhex(p["accum"]))), p


def test_sampled_pixels_c5_multi_chunk(final_scene, knobs):
    """C5 (1200x800 at 10000 spp): the rows of 8 pixels the reference
    rendered at full spp (tests/golden/make_c5.py), on a 32 MB sample buffer
    so that each row takes 4 sample chunks whose running sums continue across
    launches."""
    fx = golden("c5_pixels.json")
    w, h, spp = fx["width"], fx["height"], fx["spp"]
    cam = np.array(unhex(fx["camera"]))
    knobs("sample_buf_mb", 32)  # 1200 px x 10 B: 2796-sample chunks
    for p in fx["pixels"]:
        acc, _, st = P.render(final_scene, cam, w, h, spp, fx["max_depth"], fx["seed"],
                              row_offset=p["row"], row_stride=h)
        assert acc.shape == (1, w, 3)
        assert np.array_equal(bits(acc[0, p["i"]]), bits(unhex(p["accum"]))), p


def test_full_frames_match_reference_checksums(final_scene):
    """Full-size frames (C2 two-sphere and C3 final, 1200x800x100) against
    the reference's own full-frame checksums (tests/golden/large.json)."""
    path = os.path.join(GOLDEN, "large.json")
    if not os.path.exists(path):
        pytest.skip("large.json not generated")
    big = golden("large.json")
    cases = {"two_1200x800x100": (P.scene_two_spheres(), P.camera_default()),
             "final_1200x800x100": (final_scene, P.camera_look_at(aspect=1.5))}
    for name, (sph, cam) in cases.items():
        if name not in big:
            continue
        acc, rgb, st = P.render(sph, cam, 1200, 800, 100)
        assert sha(acc) == big[name]["accum_sha256"], name
        assert hashlib.md5(P.ppm_p3(rgb)).hexdigest() == big[name]["p3_md5"], name
        assert st["rays"] == big[name]["rays"], name


# ---- against the oracle on cases no fixture covers ---------------------------------

def test_shards_reassemble_bit_identical(oracle_mod):
    sph = oracle_mod.scene_random_spheres(1)
    cam = oracle_mod.camera_look_at(aspect=96 / 40)
    full, _, _ = P.render(sph, cam, 96, 40, 3)
    want, _, _ = oracle_mod.render(sph, cam, 96, 40, 3, threads=8)
    assert np.array_equal(bits(full), bits(want))
    for world in (2, 3, 8):
        frame = np.zeros_like(full)
        for r in range(world):
            acc, _, _ = P.render(sph, cam, 96, 40, 3, row_offset=r, row_stride=world)
            frame[r::world] = acc
        assert np.array_equal(bits(frame), bits(full)), world


def test_multi_chunk_large_spp(oracle_mod, tmp_path):
    """spp large enough to need several sample chunks on a 1 MB budget."""
    import subprocess
    import sys
    sph = oracle_mod.scene_two_spheres()
    cam = oracle_mod.camera_default()
    w, h, spp = 64, 36, 200  # 64*36*10 B = 23 KB per sample -> 44-sample chunks of 1 MB
    want, _, _ = oracle_mod.render(sph, cam, w, h, spp, threads=8)
    code = ("import numpy as np, petershirleyraytracer_amd as P;"
            "P.set_tuning('sample_buf_mb',1);"
            f"a,_,_=P.render(P.scene_two_spheres(),P.camera_default(),{w},{h},{spp});"
            f"np.save({str(tmp_path / 'c.npy')!r},a)")
    subprocess.run([sys.executable, "-c", code], check=True, cwd=ROOT, timeout=300)
    got = np.load(tmp_path / "c.npy")
    assert np.array_equal(bits(got), bits(want))


def test_units_per_launch_limit(oracle_mod, knobs):
    """A shard of more than 2^32 samples (1024 x 1024 at 4100 spp): the
    sample chunks are bounded by the 32-bit unit ids, not by the buffer, and
    balanced (2 x ~2050 samples). The frame must not depend on how the
    samples are chunked (14 chunks on a 3000 MB buffer), and its first row
    must equal the oracle's."""
    two = oracle_mod.scene_two_spheres()
    cam = oracle_mod.camera_default()
    w, h, spp = 1024, 1024, 4100
    assert w * h * spp > 2**32
    knobs("sample_buf_mb", 49152)
    big, _, st_big = P.render(two, cam, w, h, spp)
    knobs("sample_buf_mb", 3000)
    small, _, st_small = P.render(two, cam, w, h, spp)
    assert np.array_equal(bits(big), bits(small))
    assert st_big["rays"] == st_small["rays"]
    want, _, _ = oracle_mod.render(two, cam, w, h, spp, row_offset=0, row_stride=h, threads=16)
    assert np.array_equal(bits(big[:1]), bits(want))


def test_edge_cases_vs_oracle(oracle_mod):
    two = oracle_mod.scene_two_spheres()
    cam = oracle_mod.camera_default()
    for (w, h, spp, depth, seed) in [(2, 2, 1, 50, 0), (3, 2, 5, 1, 9), (17, 5, 2, 200, 3),
                                     (33, 7, 1, 50, 2**64 - 1)]:
        got, _, st = P.render(two, cam, w, h, spp, depth, seed)
        want, _, rays = oracle_mod.render(two, cam, w, h, spp, depth, seed)
        assert np.array_equal(bits(got), bits(want)), (w, h, spp, depth)
        assert st["rays"] == rays
    # empty world: every sample is sky
    got, _, st = P.render(np.zeros((0, 4)), cam, 16, 9, 2)
    want, _, _ = oracle_mod.render(np.zeros((0, 4)), cam, 16, 9, 2)
    assert np.array_equal(bits(got), bits(want))
    assert st["rays"] == 16 * 9 * 2
    # many spheres
    rng = np.random.default_rng(11)
    many = np.concatenate([rng.uniform(-5, 5, (2000, 3)), rng.uniform(0.05, 0.5, (2000, 1))], 1)
    many[:, 2] -= 8
    got, _, _ = P.render(many, cam, 24, 13, 2)
    want, _, _ = oracle_mod.render(many, cam, 24, 13, 2, threads=8)
    assert np.array_equal(bits(got), bits(want))


def test_context_device_buffers(oracle_mod):
    """rt_render_device into torch-owned HBM buffers + device quantize."""
    import torch
    sph = oracle_mod.scene_random_spheres(1)
    cam = oracle_mod.camera_look_at(aspect=64 / 40)
    ctx = P.Context(0)
    ctx.set_scene(sph, cam)
    acc = torch.zeros((40, 64, 3), dtype=torch.float64, device="cuda:0")
    rgb = torch.zeros((40, 64, 3), dtype=torch.uint8, device="cuda:0")
    stream = torch.cuda.current_stream()
    ctx.render_device(P.params(64, 40, 4), acc.data_ptr(), rgb.data_ptr(), stream.cuda_stream)
    st = ctx.sync_stats()
    torch.cuda.synchronize()
    want, wrgb, rays = oracle_mod.render(sph, cam, 64, 40, 4, threads=8)
    assert np.array_equal(bits(acc.cpu().numpy()), bits(want))
    assert np.array_equal(rgb.cpu().numpy(), wrgb)
    assert st["rays"] == rays
    rgb2 = torch.zeros_like(rgb)
    ctx.quantize_device(acc.data_ptr(), 64, 40, 4, rgb2.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(rgb2, rgb)
    ctx.close()


def test_context_repeat_renders_stats(oracle_mod):
    """Renders on one context leave its queue heads and counter sets at zero
    (psrt_reduce resets them; no memset in the render's stream): repeated
    renders, RT_FLAG_NO_TAIL_PRIORITY and a multi-chunk render all give the
    same bits and the same statistics."""
    import torch
    from petershirleyraytracer_amd.render import FLAG_CULL_STATS, FLAG_NO_TAIL_PRIORITY
    sph = oracle_mod.scene_random_spheres(1)
    cam = oracle_mod.camera_look_at(aspect=120 / 80)
    ctx = P.Context(0)
    ctx.set_scene(sph, cam)
    acc = torch.zeros((80, 120, 3), dtype=torch.float64, device="cuda:0")
    rgb = torch.zeros((80, 120, 3), dtype=torch.uint8, device="cuda:0")
    s = ctx.stream()
    keys = ("rays", "tests_executed", "box_tests", "rays_traced")
    runs = []
    C = FLAG_CULL_STATS
    for flags, buf_mb in ((C, None), (C, None), (C | FLAG_NO_TAIL_PRIORITY, None), (C, "1")):
        if buf_mb:
            ctx.set_tuning("sample_buf_mb", int(buf_mb))  # 9600 px x 10 B: 8-sample chunks
        ctx.render_device(P.params(120, 80, 300, flags=flags), acc.data_ptr(), rgb.data_ptr(), s)
        st = ctx.sync_stats()
        torch.cuda.synchronize()
        runs.append((bits(acc.cpu().numpy()), rgb.cpu().numpy(), {k: st[k] for k in keys}))
    for a, r, st in runs[1:]:
        assert np.array_equal(a, runs[0][0]) and np.array_equal(r, runs[0][1])
        assert st == runs[0][2]
    assert runs[0][2]["rays"] > 0 and runs[0][2]["box_tests"] > 0
    ctx.close()


def test_c5_row_with_hbm_nearly_full(final_scene):
    """Graceful HBM sizing: with most of the GPU's memory taken by another
    allocation (torch here), the sample buffer shrinks to what is free and
    the frame is rendered in more sample chunks, bit-identical to the
    reference's C5 pixel (tests/golden/c5_pixels.json; running sums across
    chunks, main.cc:77-84) instead of failing with RT_E_NOMEM."""
    import torch
    fx = golden("c5_pixels.json")
    w, h, spp = fx["width"], fx["height"], fx["spp"]
    cam = np.array(unhex(fx["camera"]))
    free, _ = torch.cuda.mem_get_info(0)
    # leave ~300 MB: the library keeps a 256 MiB reserve, so ~44 MB of
    # sample records (3 chunks of a 1200-pixel row at 10000 spp, 120 MB) fit
    hog = torch.empty(free - (300 << 20), dtype=torch.uint8, device="cuda:0")
    try:
        p = fx["pixels"][0]
        ctx = P.Context(0)
        ctx.set_scene(final_scene, cam)
        acc = torch.zeros((1, w, 3), dtype=torch.float64, device="cuda:0")
        ctx.render_device(P.params(w, h, spp, fx["max_depth"], fx["seed"], p["row"], h),
                          acc.data_ptr(), 0, 0)
        ctx.sync_stats()
        torch.cuda.synchronize()
        got = acc.cpu().numpy()
        ctx.close()
    finally:
        del hog
        torch.cuda.empty_cache()
    assert np.array_equal(bits(got[0, p["i"]]), bits(unhex(p["accum"]))), p


def test_hbm_nearly_full_other_buffers(final_scene, oracle_mod):
    """The sample buffer is sized after the render's other buffers:
    with ~440 MB of HBM left, (a) three chunked frames with no caller
    accumulators (a 69 MB scratch block holds their running sums) and (b) a
    material render (its path scratch: resident lanes x max_depth ints) both
    complete, bit-identical to the same renders with the GPU free."""
    import torch
    from petershirleyraytracer_amd.render import FLAG_MATERIALS, LensCamera
    w, h, spp, nf = 1200, 800, 8, 3
    cam = oracle_mod.camera_look_at(aspect=w / h)
    sp_b, mt_b = oracle_mod.scene_book_final(1)
    lens = oracle_mod.camera_look_at_lens(aspect=1.5)
    lc = LensCamera(lens["base"], lens["u"], lens["v"], lens["lens_radius"])
    mw, mh, mspp = 480, 320, 48

    def frames(ctx):
        rgb = [torch.zeros((h, w, 3), dtype=torch.uint8, device="cuda:0") for _ in range(nf)]
        ctx.render_device_frames(P.params(w, h, spp, 50, 5), nf, None, [r.data_ptr() for r in rgb])
        ctx.sync_stats()
        torch.cuda.synchronize()
        return [r.cpu().numpy() for r in rgb]

    def mat(ctx):
        acc = torch.zeros((mh, mw, 3), dtype=torch.float64, device="cuda:0")
        ctx.render_device(P.params(mw, mh, mspp, 50, 3, flags=FLAG_MATERIALS), acc.data_ptr())
        ctx.sync_stats()
        torch.cuda.synchronize()
        return acc.cpu().numpy()

    def run(hog_left):
        hog = None
        if hog_left:
            free, _ = torch.cuda.mem_get_info(0)
            hog = torch.empty(free - hog_left, dtype=torch.uint8, device="cuda:0")
        try:
            c1 = P.Context(0)
            c1.set_scene(final_scene, cam)
            a = frames(c1)
            c1.close()
            c2 = P.Context(0)
            c2.set_scene(sp_b, lens["base"])
            c2.set_materials(mt_b, lc)
            b = mat(c2)
            c2.close()
        finally:
            del hog
            torch.cuda.empty_cache()
        return a, b

    want_f, want_m = run(0)
    got_f, got_m = run(440 << 20)
    for f in range(nf):
        assert np.array_equal(got_f[f], want_f[f]), f
    assert np.array_equal(bits(got_m), bits(want_m))
