"""Materials and defocus — CPU side.

The reference has no materials (its ray_color is the 0.5-attenuation
hemisphere bounce of main.cc:42-43), so nothing here can be pinned to the
reference's output: parity unpinned. What is pinned:
  * the C restatement (oracle/rt_oracle_mat.c) against an independently
    written pure-Python restatement (tests/mat_pyref.py), bit for bit;
  * the product's host helpers (book scene, lens camera) against the oracle's;
  * the oracle's own invariants (thread count, shards, depth edges).
The GPU tests (test_gpu_materials.py) then compare the device with the oracle.
"""
import numpy as np
import pytest

from conftest import bits

import mat_pyref

# A small scene with every material case: lambertian ground and sphere, a
# hollow glass sphere (negative radius inside, the book's ch. 10.5 trick),
# polished and fuzzy metal, and a metal whose fuzz is clamped to 1.
MIXED_SPHERES = np.array([
    [0.0, -100.5, -1.0, 100.0],
    [0.0, 0.0, -1.0, 0.5],
    [-1.0, 0.0, -1.0, 0.5],
    [-1.0, 0.0, -1.0, -0.45],
    [1.0, 0.0, -1.0, 0.5],
    [0.35, -0.35, -0.55, 0.12],
    [-0.3, -0.38, -0.45, 0.1],
])
MIXED_MATS = np.array([
    [0, 0.8, 0.8, 0.0, 0.0, 0.0],
    [0, 0.1, 0.2, 0.5, 0.0, 0.0],
    [2, 1.0, 1.0, 1.0, 0.0, 1.5],
    [2, 1.0, 1.0, 1.0, 0.0, 1.5],
    [1, 0.8, 0.6, 0.2, 0.0, 0.0],
    [1, 0.7, 0.7, 0.9, 1.7, 0.0],
    [1, 0.9, 0.5, 0.4, 0.3, 0.0],
])


def mixed_lens(oracle, aperture=0.1, aspect=1.5):
    return oracle.camera_look_at_lens((-2, 2, 1), (0, 0, -1), (0, 1, 0), 20.0, aspect, aperture,
                                      3.4)


def test_oracle_matches_python_restatement(oracle_mod):
    lens = mixed_lens(oracle_mod)
    W, H, spp, depth, seed = 9, 6, 3, 12, 5
    acc, rays = oracle_mod.render_mat(MIXED_SPHERES, MIXED_MATS, lens, W, H, spp, depth, seed)
    ref = mat_pyref.render_mat(MIXED_SPHERES, MIXED_MATS, lens, W, H, spp, depth, seed, oracle_mod)
    assert np.array_equal(bits(acc), bits(ref))
    assert rays >= W * H * spp


def test_oracle_matches_python_restatement_book_scene(oracle_mod):
    """The book's final scene, lens on: a handful of pixels near the centre."""
    sp, mt = oracle_mod.scene_book_final(1)
    lens = oracle_mod.camera_look_at_lens(aspect=1.5)
    W, H = 12, 8
    acc, _ = oracle_mod.render_mat(sp, mt, lens, W, H, 1, 50, 11)
    ref = mat_pyref.render_mat(sp, mt, lens, W, H, 1, 50, 11, oracle_mod)
    assert np.array_equal(bits(acc), bits(ref))


def test_book_scene_and_lens_camera_match_oracle(oracle_mod):
    import petershirleyraytracer_amd as P
    for seed in (1, 7):
        sp, mt = P.scene_book_final(seed)
        osp, omt = oracle_mod.scene_book_final(seed)
        assert np.array_equal(bits(sp), bits(osp)) and np.array_equal(bits(mt), bits(omt))
    sp, mt = P.scene_book_final(1)
    kinds = np.bincount(mt[:, 0].astype(int), minlength=3)
    assert len(sp) == 487 and tuple(kinds) == (394, 64, 29)
    assert (mt[mt[:, 0] == 1, 4] <= 0.5).all()  # metal fuzz = random_double(0, 0.5)
    for args in [dict(), dict(aperture=0.0, focus_dist=1.0), dict(lookfrom=(3, 3, 2),
                 lookat=(0, 0, -1), vfov=20.0, aspect=2.0, aperture=2.0, focus_dist=5.2)]:
        a = P.camera_look_at_lens(**args)
        b = oracle_mod.camera_look_at_lens(**args)
        assert np.array_equal(bits(a.base), bits(b["base"]))
        assert np.array_equal(bits(a.u), bits(b["u"])) and np.array_equal(bits(a.v), bits(b["v"]))
        assert a.lens_radius == b["lens_radius"]
    # aperture 0, focus distance 1: the pinhole look-at camera
    assert np.array_equal(bits(P.camera_look_at_lens(aperture=0.0, focus_dist=1.0).base),
                          bits(P.camera_look_at()))


def test_oracle_threads_and_shards(oracle_mod):
    lens = mixed_lens(oracle_mod)
    W, H = 20, 13
    a1, r1 = oracle_mod.render_mat(MIXED_SPHERES, MIXED_MATS, lens, W, H, 4, 20, 3, threads=1)
    a4, r4 = oracle_mod.render_mat(MIXED_SPHERES, MIXED_MATS, lens, W, H, 4, 20, 3, threads=4)
    assert np.array_equal(bits(a1), bits(a4)) and r1 == r4
    rays = 0
    for off in range(3):
        part, r = oracle_mod.render_mat(MIXED_SPHERES, MIXED_MATS, lens, W, H, 4, 20, 3, off, 3)
        assert np.array_equal(bits(part), bits(a1[off::3]))
        rays += r
    assert rays == r1


def test_oracle_depth_edges(oracle_mod):
    lens = mixed_lens(oracle_mod)
    for d in (0, -1):
        acc, rays = oracle_mod.render_mat(MIXED_SPHERES, MIXED_MATS, lens, 8, 5, 2, d, 0)
        assert rays == 0 and not acc.any()
    with pytest.raises(RuntimeError):
        oracle_mod.render_mat(MIXED_SPHERES, MIXED_MATS, lens, 8, 5, 2, 4097, 0)
    # depth 1: a miss is the sky, any hit is black
    acc, rays = oracle_mod.render_mat(MIXED_SPHERES, MIXED_MATS, lens, 8, 5, 1, 1, 0)
    assert rays == 40


def test_material_symbols_exported():
    import petershirleyraytracer_amd._lib as L
    lib = L.load()
    for name in ("rt_camera_look_at_lens", "rt_scene_book_final", "rt_context_set_materials",
                 "rt_render_materials"):
        assert hasattr(lib, name)
