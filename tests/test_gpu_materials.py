"""Materials and defocus on the device (psrt_trace_mat).

Bit-exact against oracle/rt_oracle_mat.c (pinned to tests/mat_pyref.py by
test_materials.py). Parity with the reference itself is unpinned: the
reference has no materials.
"""
import os

import numpy as np
import pytest

from conftest import bits

import petershirleyraytracer_amd as P
from petershirleyraytracer_amd import _lib
from petershirleyraytracer_amd.render import FLAG_MATERIALS, FLAG_NO_CULL, LensCamera
from test_materials import MIXED_MATS, MIXED_SPHERES, mixed_lens

pytestmark = pytest.mark.gpu


def _lens(d) -> LensCamera:
    return LensCamera(d["base"], d["u"], d["v"], d["lens_radius"])


@pytest.fixture(scope="module")
def book(oracle_mod):
    sp, mt = oracle_mod.scene_book_final(1)
    return sp, mt, oracle_mod.camera_look_at_lens(aspect=1.5)


@pytest.mark.parametrize("cull,lds", [(True, None), (True, "0"), (False, None)])
def test_book_scene_bit_exact(oracle_mod, book, cull, lds, knobs):
    """The culled kernel with the scene in LDS (default) and in global memory
    (tuning knob mat_lds = 0), and the linear scan."""
    if lds is not None:
        knobs("mat_lds", int(lds))
    sp, mt, lens = book
    W, H, spp, seed = 72, 48, 4, 9
    acc, rgb, st = P.render_materials(sp, mt, _lens(lens), W, H, spp, 50, seed, cull=cull)
    ref, rays = oracle_mod.render_mat(sp, mt, lens, W, H, spp, 50, seed, threads=8)
    assert np.array_equal(bits(acc), bits(ref))
    assert np.array_equal(rgb, oracle_mod.quantize(ref, spp))
    assert st["rays"] == rays and st["samples"] == W * H * spp


def test_mixed_scene_bit_exact(oracle_mod):
    lens = mixed_lens(oracle_mod)
    W, H, spp, seed = 60, 40, 6, 2
    acc, rgb, st = P.render_materials(MIXED_SPHERES, MIXED_MATS, _lens(lens), W, H, spp, 30, seed)
    ref, rays = oracle_mod.render_mat(MIXED_SPHERES, MIXED_MATS, lens, W, H, spp, 30, seed,
                                      threads=8)
    assert np.array_equal(bits(acc), bits(ref))
    assert st["rays"] == rays


def test_shards_and_depth_edges(oracle_mod, book):
    sp, mt, lens = book
    W, H, spp = 40, 27, 2
    full, _ = oracle_mod.render_mat(sp, mt, lens, W, H, spp, 8, 4, threads=8)
    for off in range(3):
        acc, _, _ = P.render_materials(sp, mt, _lens(lens), W, H, spp, 8, 4, off, 3)
        assert np.array_equal(bits(acc), bits(full[off::3]))
    for d in (0, -1):
        acc, rgb, st = P.render_materials(sp, mt, _lens(lens), W, H, spp, d, 4)
        assert not acc.any() and not rgb.any() and st["rays"] == 0
    with pytest.raises(_lib.RtError):
        P.render_materials(sp, mt, _lens(lens), W, H, spp, 4097, 4)


def test_chunked_multi_frame_context(oracle_mod, book, knobs):
    """Sample chunks (a small buffer cap) and multi-frame launches through the
    context: frame f equals the one-shot render of seed + f."""
    import torch
    sp, mt, lens = book
    W, H, spp, seed, nf = 32, 20, 48, 21, 3
    # 1 MiB holds 22 samples of 3 frames x 640 pixels x 24 B: 3 chunks of 16
    knobs("sample_buf_mb", 1)
    ctx = P.Context(0)
    try:
        ctx.set_scene(sp, lens["base"])
        with pytest.raises(_lib.RtError):  # no materials yet
            ctx.render_device(P.params(W, H, spp, 50, seed, flags=FLAG_MATERIALS))
        ctx.set_materials(mt, _lens(lens))
        acc = [torch.zeros((H, W, 3), dtype=torch.float64, device="cuda") for _ in range(nf)]
        rgb = [torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda") for _ in range(nf)]
        ctx.render_device_frames(P.params(W, H, spp, 50, seed, flags=FLAG_MATERIALS), nf,
                                 [a.data_ptr() for a in acc], [r.data_ptr() for r in rgb])
        st = ctx.sync_stats()
        total = 0
        for f in range(nf):
            ref, rays = oracle_mod.render_mat(sp, mt, lens, W, H, spp, 50, seed + f, threads=8)
            assert np.array_equal(bits(acc[f].cpu().numpy()), bits(ref)), f
            assert np.array_equal(rgb[f].cpu().numpy(), oracle_mod.quantize(ref, spp)), f
            total += rays
        assert st["rays"] == total
        # the same context, back to the reference integrator: unchanged bits
        ctx.render_device(P.params(W, H, spp, 50, seed), acc[0].data_ptr())
        ctx.sync_stats()
        ref, _, _ = oracle_mod.render(sp, lens["base"], W, H, spp, 50, seed, threads=8)
        assert np.array_equal(bits(acc[0].cpu().numpy()), bits(ref))
    finally:
        ctx.close()


def test_lens_radius_zero_and_no_cull_flag(oracle_mod):
    lens = mixed_lens(oracle_mod, aperture=0.0)
    W, H, spp = 30, 20, 3
    a, _, _ = P.render_materials(MIXED_SPHERES, MIXED_MATS, _lens(lens), W, H, spp, 50, 1,
                                 cull=False)
    ref, _ = oracle_mod.render_mat(MIXED_SPHERES, MIXED_MATS, lens, W, H, spp, 50, 1, threads=8)
    assert np.array_equal(bits(a), bits(ref))
    assert FLAG_NO_CULL == 1


def test_long_paths_between_mirrors(oracle_mod):
    """Paths that use the path column deeply: two near-parallel mirror spheres
    (r = 1e5, a gap of 1) with glass and diffuse balls between them; ~76 rays
    per sample, some paths cut at depth 300; the same at depth 4096 (the
    RT_FLAG_MATERIALS bound)."""
    R = 1e5
    sp = np.array([[0, -R - 0.5, 0, R], [0, R + 0.5, 0, R], [0.0, 0.0, -3.0, 0.25],
                   [0.4, 0.1, -6.0, 0.3], [-0.5, -0.1, -9.0, -0.2]])
    mt = np.array([[1, 0.98, 0.97, 0.96, 0.0, 0.0], [1, 0.97, 0.98, 0.99, 0.02, 0.0],
                   [2, 1, 1, 1, 0.0, 1.5], [0, 0.7, 0.3, 0.2, 0, 0], [2, 1, 1, 1, 0, 1.5]])
    lens = oracle_mod.camera_look_at_lens((0, 0, 0), (0, 0.05, -1), (0, 1, 0), 60.0, 4 / 3, 0.0,
                                          1.0)
    for depth in (300, 4096):
        acc, _, st = P.render_materials(sp, mt, _lens(lens), 16, 12, 3, depth, 5)
        ref, rays = oracle_mod.render_mat(sp, mt, lens, 16, 12, 3, depth, 5, threads=8)
        assert np.array_equal(bits(acc), bits(ref)), depth
        assert st["rays"] == rays and rays > 50 * 16 * 12 * 3


@pytest.mark.parametrize("aperture", [0.1, 2.0, 0.0])
def test_apertures_bit_exact(oracle_mod, book, knobs, aperture):
    """The book's aperture, a wide one and a pinhole, at 240 x 160 x 6.
    Camera rays through the lens test only their pixel's candidate list
    (psrt_mat_camera_lists): the frame equals the one without
    lists (tuning knob no_camlist) bit for bit, and the oracle's."""
    sp, mt, _ = book
    W, H, spp = 240, 160, 6
    lens = oracle_mod.camera_look_at_lens(aspect=W / H, aperture=aperture)
    acc, rgb, st = P.render_materials(sp, mt, _lens(lens), W, H, spp, 50, 13)
    knobs("no_camlist", 1)
    acc2, _, st2 = P.render_materials(sp, mt, _lens(lens), W, H, spp, 50, 13)
    assert np.array_equal(bits(acc), bits(acc2)) and st["rays"] == st2["rays"]
    ref, rays = oracle_mod.render_mat(sp, mt, lens, W, H, spp, 50, 13, threads=8)
    assert np.array_equal(bits(acc), bits(ref)) and st["rays"] == rays
    assert np.array_equal(rgb, oracle_mod.quantize(ref, spp))


def test_cli_book_scene(oracle_mod, tmp_path):
    """bin/raytracer --scene book: the book scene through psrt::render_materials
    (include/psrt/render.hpp), P3 text equal to the oracle's frame quantised."""
    import subprocess
    from conftest import ROOT
    exe = os.path.join(ROOT, "petershirleyraytracer_amd", "bin", "raytracer")
    out = tmp_path / "book.ppm"
    subprocess.run([exe, "--scene", "book", "--width", "48", "--height", "32", "--spp", "3",
                    "--seed", "4", "-o", str(out)], check=True, timeout=120, capture_output=True)
    sp, mt = oracle_mod.scene_book_final(1)
    lens = oracle_mod.camera_look_at_lens(aspect=48 / 32)
    ref, _ = oracle_mod.render_mat(sp, mt, lens, 48, 32, 3, 50, 4, threads=8)
    assert out.read_bytes() == oracle_mod.ppm_p3(oracle_mod.quantize(ref, 3))


def test_counting_variant_same_bits(oracle_mod, book):
    """RT_FLAG_CULL_STATS selects the material kernel that counts its sphere /
    box tests: the same frame, non-zero counts (zero without the flag)."""
    import torch
    from petershirleyraytracer_amd.render import FLAG_CULL_STATS
    sp, mt, lens = book
    W, H, spp = 64, 40, 4
    ctx = P.Context(0)
    try:
        ctx.set_scene(sp, lens["base"])
        ctx.set_materials(mt, _lens(lens))
        out = []
        for fl in (0, FLAG_CULL_STATS):
            acc = torch.zeros((H, W, 3), dtype=torch.float64, device="cuda")
            ctx.render_device(P.params(W, H, spp, 50, 3, flags=FLAG_MATERIALS | fl), acc.data_ptr())
            out.append((acc.cpu().numpy(), ctx.sync_stats()))
        assert np.array_equal(bits(out[0][0]), bits(out[1][0]))
        assert out[0][1]["tests_executed"] == 0 and out[1][1]["tests_executed"] > out[1][1]["rays"]
        assert out[1][1]["box_tests"] > 0 and out[0][1]["rays"] == out[1][1]["rays"]
    finally:
        ctx.close()


def test_failure_hook_on_the_material_path(oracle_mod, book):
    """rt_debug_fail_after_trace fails a RT_FLAG_MATERIALS render after its
    trace launch, as it does the reference integrator's (the hook
    was consumed silently); the next render is whole and bit-exact."""
    import torch
    sp, mt, lens = book
    W, H, spp = 40, 24, 3
    ctx = P.Context(0)
    try:
        ctx.set_scene(sp, lens["base"])
        ctx.set_materials(mt, _lens(lens))
        acc = torch.zeros((H, W, 3), dtype=torch.float64, device="cuda")
        ctx.debug_fail_after_trace(0)
        with pytest.raises(_lib.RtError, match="injected"):
            ctx.render_device(P.params(W, H, spp, 50, 6, flags=FLAG_MATERIALS), acc.data_ptr())
        failed = ctx.sync_stats()
        assert failed["rays"] == 0 and failed["kernel_ms"] == 0.0
        ctx.render_device(P.params(W, H, spp, 50, 6, flags=FLAG_MATERIALS), acc.data_ptr())
        st = ctx.sync_stats()
        torch.cuda.synchronize()
        ref, rays = oracle_mod.render_mat(sp, mt, lens, W, H, spp, 50, 6, threads=8)
        assert np.array_equal(bits(acc.cpu().numpy()), bits(ref)) and st["rays"] == rays
    finally:
        ctx.close()


def _contact_mat_scene(rng):
    """Touching, nested and hollow spheres on a ground and against a second
    big sphere standing as a wall: the direction lists' cell keys (two big
    surfaces) and sphere keys (rays leaving a sphere into its neighbours, or
    back into itself through glass) at their tightest."""
    sp = [[0.0, -1000.0, 0.0, 1000.0], [-504.0, 0.0, 0.0, 500.0]]
    mt = [[0, 0.5, 0.5, 0.5, 0, 0], [1, 0.8, 0.8, 0.9, 0.05, 0]]
    for _ in range(60):
        r = rng.uniform(0.1, 0.5)
        c = [rng.uniform(-3.5, 3), r, rng.uniform(-3, 3)]
        sp.append(c + [r])
        kind = rng.integers(0, 3)
        mt.append([kind, *rng.uniform(0.2, 0.9, 3), rng.uniform(0, 0.3), 1.5])
        if rng.random() < 0.3:  # a touching neighbour / a hollow shell inside glass
            d = rng.normal(size=3)
            d /= np.linalg.norm(d)
            r2 = rng.uniform(0.05, 0.3)
            sp.append([c[0] + d[0] * (r + r2), max(r2, c[1] + d[1] * (r + r2)), c[2] + d[2] * (r + r2), r2])
            mt.append([rng.integers(0, 3), 0.6, 0.6, 0.6, 0.1, 1.5])
        if kind == 2 and rng.random() < 0.5:
            sp.append(c + [-0.9 * r])
            mt.append([2, 1, 1, 1, 0, 1.5])
    return np.array(sp), np.array(mt, dtype=float)


def test_contact_scenes_two_big_surfaces(oracle_mod):
    """Touching, nested and hollow spheres between a ground and a second big
    sphere standing as a wall (the scenes the r05 direction-list experiment
    was checked on, profiles/r05_dirlist): frames equal the oracle's."""
    for seed in (1, 2):
        s, m = _contact_mat_scene(np.random.default_rng(seed))
        lens = oracle_mod.camera_look_at_lens((3.0, 2.0, 6.0), (0.0, 0.3, 0.0), (0, 1, 0), 50.0,
                                              1.5, 0.05, 6.0)
        acc, _, st = P.render_materials(s, m, _lens(lens), 90, 60, 4, 50, 7)
        ref, rays = oracle_mod.render_mat(s, m, lens, 90, 60, 4, 50, 7, threads=8)
        assert np.array_equal(bits(acc), bits(ref)) and st["rays"] == rays, seed
