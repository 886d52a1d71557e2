"""Randomised scene sweep (r05): seeded random worlds and cameras through the
culled kernels (BVH, grid, neighbour and camera lists, the §9 fixed-point
exit; the material integrator's lists and walk) against the C oracle, bit for
bit, with the reference's ray counts. The worlds vary what the exactness
arguments lean on: sphere counts around the BVH threshold and far above it,
flat layers, clusters with touching and duplicate spheres, negative radii,
tiny and huge radii, a big ground or none, cameras inside the cloud and far
out, fields of view from 5 to 120 degrees."""
import numpy as np
import pytest

from conftest import bits

import petershirleyraytracer_amd as P
from petershirleyraytracer_amd.render import LensCamera

pytestmark = pytest.mark.gpu


def _world(rng):
    n = int(rng.choice([17, 40, 150, 600, 1500]))
    kind = rng.integers(0, 4)
    if kind == 0:    # uniform cube
        c = rng.uniform(-6, 6, (n, 3))
        r = rng.uniform(0.05, 0.8, n)
    elif kind == 1:  # flat layer on the ground (the final scene's shape)
        c = np.stack([rng.uniform(-11, 11, n), np.zeros(n), rng.uniform(-11, 11, n)], 1)
        r = rng.uniform(0.1, 0.3, n)
        c[:, 1] = r
    elif kind == 2:  # clusters: touching pairs and duplicates
        base = rng.uniform(-4, 4, (n // 2, 3))
        rb = rng.uniform(0.1, 0.6, n // 2)
        d = rng.normal(size=base.shape)
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        r2 = rng.uniform(0.05, 0.5, n // 2)
        dup = rng.random(n // 2) < 0.2
        c = np.concatenate([base, np.where(dup[:, None], base, base + d * (rb + r2)[:, None])])
        r = np.concatenate([rb, np.where(dup, rb, r2)])
    else:            # mixed scales
        c = rng.uniform(-20, 20, (n, 3))
        r = np.exp(rng.uniform(np.log(1e-3), np.log(3.0), n))
    r = np.where(rng.random(len(r)) < 0.05, -r, r)  # a few negative radii (hollow shells)
    sph = np.concatenate([c, r[:, None]], 1)
    if rng.random() < 0.7:  # a big ground
        sph = np.concatenate([[[0.0, -1000.0, 0.0, 1000.0]], sph])
    return sph


def _camera(rng, aspect):
    look_from = rng.normal(size=3) * rng.choice([3.0, 15.0, 60.0])
    look_at = rng.normal(size=3) * 2.0
    if np.linalg.norm(look_from - look_at) < 0.5:
        look_from = look_at + np.array([0.0, 1.0, 5.0])
    return P.camera_look_at(tuple(look_from), tuple(look_at), vfov=float(rng.uniform(5, 120)),
                            aspect=aspect)


@pytest.mark.parametrize("seed", range(64))
def test_random_worlds_reference_integrator(oracle_mod, seed):
    rng = np.random.default_rng(1000 + seed)
    sph = _world(rng)
    W, H, spp = 48, 32, 4
    cam = _camera(rng, W / H)
    depth = int(rng.choice([3, 50, 50]))
    s = int(rng.integers(0, 2**31))
    acc, rgb, st = P.render(sph, cam, W, H, spp, depth, s)
    ref, rref, rays = oracle_mod.render(sph, cam, W, H, spp, depth, s, threads=8)
    assert np.array_equal(bits(acc), bits(ref)), (seed, len(sph))
    assert np.array_equal(rgb, rref) and st["rays"] == rays, seed


@pytest.mark.parametrize("seed", range(24))
def test_random_worlds_materials(oracle_mod, seed):
    rng = np.random.default_rng(2000 + seed)
    sph = _world(rng)
    n = len(sph)
    kinds = rng.integers(0, 3, n)
    mats = np.concatenate([kinds[:, None], rng.uniform(0.1, 0.95, (n, 3)),
                           rng.uniform(0.0, 1.2, (n, 1)), rng.uniform(1.1, 2.4, (n, 1))], 1)
    W, H, spp = 40, 30, 3
    look_from = rng.normal(size=3) * rng.choice([4.0, 15.0])
    lens = oracle_mod.camera_look_at_lens(tuple(look_from), (0.0, 0.0, 0.0), (0, 1, 0),
                                          float(rng.uniform(10, 90)), W / H,
                                          float(rng.choice([0.0, 0.1, 1.0])),
                                          float(rng.uniform(2, 20)))
    s = int(rng.integers(0, 2**31))
    acc, _, st = P.render_materials(sph, mats, LensCamera(lens["base"], lens["u"], lens["v"],
                                                          lens["lens_radius"]), W, H, spp, 50, s)
    ref, rays = oracle_mod.render_mat(sph, mats, lens, W, H, spp, 50, s, threads=8)
    assert np.array_equal(bits(acc), bits(ref)), (seed, n)
    assert st["rays"] == rays, seed
