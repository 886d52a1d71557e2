"""Exact culling: the BVH path must return exactly what the
reference's linear list scan returns — same index, same record bits — for
every ray, and whole renders must stay bit-identical to the oracle/reference."""
import numpy as np
import pytest

from conftest import bits, golden, sha, unhex

import petershirleyraytracer_amd as P
from petershirleyraytracer_amd.render import world_hit

pytestmark = pytest.mark.gpu


def _rays_on_surfaces(sph, n, rng):
    idx = rng.integers(0, len(sph), n)
    v = rng.normal(size=(n, 3))
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    o = sph[idx, :3] + sph[idx, 3:4] * v
    d = rng.normal(size=(n, 3))
    return o, d


def _tangent_rays(sph, n, rng):
    """Rays that graze a random sphere (distance to centre ~ r +- tiny)."""
    idx = rng.integers(0, len(sph), n)
    c, r = sph[idx, :3], sph[idx, 3]
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    perp = rng.normal(size=(n, 3))
    perp -= (perp * d).sum(1, keepdims=True) * d
    perp /= np.linalg.norm(perp, axis=1, keepdims=True)
    eps = rng.choice([0.0, 1e-15, -1e-15, 1e-9, -1e-9, 1e-6], n)
    p = c + (r * (1 + eps))[:, None] * perp
    back = rng.uniform(0.0, 30.0, n)[:, None]
    o = p - back * d
    return o, d * rng.uniform(0.1, 3.0, (n, 1))


def _compare(sph, o, d):
    rays = np.concatenate([o, d, np.zeros((len(o), 1)), np.full((len(o), 1), np.inf)], 1)
    a = world_hit(sph, rays, cull=True)
    b = world_hit(sph, rays, cull=False)
    same = (bits(a) == bits(b)) | (np.isnan(a) & np.isnan(b))
    bad = np.where(~same.all(1))[0]
    assert len(bad) == 0, (len(bad), rays[bad[:3]], a[bad[:3]], b[bad[:3]])
    return (a[:, 0] >= 0).mean()


def test_bvh_equals_linear_final_scene(final_scene):
    rng = np.random.default_rng(123)
    n = 400_000
    hit_rate = []
    o, d = _rays_on_surfaces(final_scene, n, rng)
    hit_rate.append(_compare(final_scene, o, d))
    o, d = _tangent_rays(final_scene, n, rng)
    hit_rate.append(_compare(final_scene, o, d))
    o = rng.uniform(-15, 15, (n, 3))
    o[:, 1] = rng.uniform(-0.5, 3, n)
    hit_rate.append(_compare(final_scene, o, rng.normal(size=(n, 3))))
    # far origins (beyond r_check some take the linear path) aimed at the scene
    o = rng.normal(size=(n, 3)) * rng.choice([50.0, 500.0, 3000.0], (n, 1))
    d = rng.uniform(-3, 3, (n, 3)) - o
    hit_rate.append(_compare(final_scene, o, d))
    # camera rays of the bench configuration
    cam = P.camera_look_at(aspect=1.5)
    u, v = rng.uniform(0, 1, n), rng.uniform(0, 1, n)
    d = cam[1] + u[:, None] * cam[2] + v[:, None] * cam[3] - cam[0]
    hit_rate.append(_compare(final_scene, np.broadcast_to(cam[0], (n, 3)).copy(), d))
    # short segments among the small spheres: rays that meet the ground 0.02-2
    # units away, so [o, o + t d] crosses zero, one or several grid cell
    # boundaries (single-cell lists, 2x2x2 block lists, the walk)
    o = np.stack([rng.uniform(-12, 12, n), rng.uniform(1e-4, 0.6, n), rng.uniform(-12, 12, n)], 1)
    reach = rng.uniform(0.02, 2.0, n)
    ang = rng.uniform(0, 2 * np.pi, n)
    d = np.stack([reach * np.cos(ang), -o[:, 1], reach * np.sin(ang)], 1)
    hit_rate.append(_compare(final_scene, o, d * rng.uniform(0.5, 2.0, (n, 1))))
    assert all(0.05 < h <= 1.0 for h in hit_rate), hit_rate


def test_bvh_ties_and_degenerate_scenes():
    rng = np.random.default_rng(5)
    base = np.concatenate([rng.uniform(-3, 3, (300, 3)), rng.uniform(0.05, 0.6, (300, 1))], 1)
    scenes = {
        "duplicates": np.concatenate([base, base[::-1]]),  # every hit is a tie
        "touching": np.array([[x, 0.0, z, 0.5] for x in range(-6, 7) for z in range(-6, 7)]),
        "nested": np.concatenate([base, base * [1, 1, 1, 0.5], base * [1, 1, 1, 0.25]]),
        "mixed_big": np.concatenate([base, [[0, -1000, 0, 1000], [0, 0, 0, 40.0],
                                            [5, 5, 5, 1e-9]]]),
        # tall spheres (3-16x the median radius): the BVH's own root subtree
        "tall": np.concatenate([base, np.concatenate([rng.uniform(-3, 3, (12, 3)),
                                                      rng.uniform(1.2, 4.0, (12, 1))], 1)]),
        "negative_r": base * [1, 1, 1, -1],
        "coincident": np.tile([[0.0, 0.0, 0.0, 1.0]], (40, 1)),
    }
    for name, sph in scenes.items():
        n = 100_000
        o, d = _rays_on_surfaces(sph, n, rng)
        _compare(sph, o, d)
        o, d = _tangent_rays(sph, n, rng)
        _compare(sph, o, d)
        o = rng.uniform(-8, 8, (n, 3))
        _compare(sph, o, rng.normal(size=(n, 3)))


def _compare_hinted(sph, o, d, hint):
    """The trace kernel's bounce-ray call (previous hit as the hint: the
    hint-first test and the neighbour-list path) against the
    reference scan."""
    rays = np.concatenate([o, d, np.zeros((len(o), 1)), np.full((len(o), 1), np.inf)], 1)
    a = world_hit(sph, rays, cull=True, hints=hint)
    b = world_hit(sph, rays, cull=False)
    same = (bits(a) == bits(b)) | (np.isnan(a) & np.isnan(b))
    bad = np.where(~same.all(1))[0]
    assert len(bad) == 0, (len(bad), rays[bad[:3]], hint[bad[:3]], a[bad[:3]], b[bad[:3]])
    return (a[:, 0] >= 0).mean()


def _bounce_rays(sph, idx, rng, mode):
    """Origins on (or within a few ulp / ~pad/8 of) sphere idx's surface;
    directions: the reference's scatter n + random_in_hemisphere(n), uniform,
    or aimed at the silhouette of another sphere (tangent +- tiny)."""
    n = len(idx)
    c, r = sph[idx, :3], np.abs(sph[idx, 3])
    u = rng.normal(size=(n, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    scale = max(1.0, float(np.max(np.abs(sph[:, :3]) + np.abs(sph[:, 3:4]))))
    off = rng.choice([0.0, 1e-16, -1e-16, 1e-12, -1e-12, 2e-5 * scale / 64, -2e-5 * scale / 64], n)
    o = c + (r * (1 + off))[:, None] * u
    if mode == "scatter":
        v = rng.uniform(-1, 1, (n, 3))
        v /= np.maximum(1.0, np.linalg.norm(v, axis=1, keepdims=True))
        v = np.where(((v * u).sum(1) > 0)[:, None], v, -v)
        return o, u + v
    if mode == "uniform":
        return o, rng.normal(size=(n, 3))
    k = rng.integers(0, len(sph), n)  # silhouette of sphere k seen from o
    ck, rk = sph[k, :3], np.abs(sph[k, 3])
    w = ck - o
    w /= np.maximum(np.linalg.norm(w, axis=1, keepdims=True), 1e-300)
    perp = rng.normal(size=(n, 3))
    perp -= (perp * w).sum(1, keepdims=True) * w
    perp /= np.maximum(np.linalg.norm(perp, axis=1, keepdims=True), 1e-300)
    eps = rng.choice([0.0, 1e-12, -1e-12, 1e-7, -1e-7, 1e-4], n)
    return o, (ck + (rk * (1 + eps))[:, None] * perp) - o


def test_hinted_bounce_rays_equal_linear(final_scene):
    """Bounce rays with their previous hit as the hint: on every BVH sphere
    and on the ground near the field, scatter / uniform / silhouette-grazing
    directions."""
    rng = np.random.default_rng(77)
    n = 300_000
    for mode in ("scatter", "uniform", "silhouette"):
        idx = rng.integers(0, len(final_scene), n)
        idx[: n // 3] = 0  # the ground (a big sphere: no neighbour list)
        o, d = _bounce_rays(final_scene, idx, rng, mode)
        if mode != "silhouette":  # ground points near the sphere field
            m = idx == 0
            g = np.stack([rng.uniform(-13, 13, m.sum()), np.zeros(m.sum()),
                          rng.uniform(-13, 13, m.sum())], 1)
            g[:, 1] = -1000.0 + np.sqrt(1000.0 ** 2 - g[:, 0] ** 2 - g[:, 2] ** 2)
            o[m] = g
            if mode == "scatter":  # n + random_in_hemisphere(n) about the ground normal
                ng = (g - [0.0, -1000.0, 0.0]) / 1000.0
                v = rng.uniform(-1, 1, (m.sum(), 3))
                v /= np.maximum(1.0, np.linalg.norm(v, axis=1, keepdims=True))
                v = np.where(((v * ng).sum(1) > 0)[:, None], v, -v)
                d[m] = ng + v
        _compare_hinted(final_scene, o, d, idx)


def test_hinted_bounce_rays_contact_scenes():
    rng = np.random.default_rng(78)
    base = np.concatenate([rng.uniform(-3, 3, (300, 3)), rng.uniform(0.05, 0.6, (300, 1))], 1)
    scenes = {
        "duplicates": np.concatenate([base, base[::-1]]),
        "touching": np.array([[x, 0.0, z, 0.5] for x in range(-6, 7) for z in range(-6, 7)]),
        "nested": np.concatenate([base, base * [1, 1, 1, 0.5], base * [1, 1, 1, 0.25]]),
        "mixed_big": np.concatenate([base, [[0, -1000, 0, 1000], [0, 0, 0, 40.0],
                                            [5, 5, 5, 1e-9]]]),
        "tall": np.concatenate([base, np.concatenate([rng.uniform(-3, 3, (12, 3)),
                                                      rng.uniform(1.2, 4.0, (12, 1))], 1)]),
        "negative_r": base * [1, 1, 1, -1],
        "sparse": np.concatenate([rng.uniform(-40, 40, (60, 3)), rng.uniform(0.2, 1.0, (60, 1))], 1),
    }
    for name, sph in scenes.items():
        for mode in ("scatter", "uniform", "silhouette"):
            idx = rng.integers(0, len(sph), 60_000)
            o, d = _bounce_rays(sph, idx, rng, mode)
            _compare_hinted(sph, o, d, idx)


def test_far_origins_inside_a_huge_ground():
    """Origins deep inside a ground sphere 10^4-10^5 scene scales big, aimed
    at small spheres half sunk into its surface: the FP32 grid query is not
    precise there, so these rays must take the guarded FP64 paths."""
    rng = np.random.default_rng(17)
    small = np.stack([rng.uniform(-3, 3, 300), rng.uniform(-0.2, 0.2, 300),
                      rng.uniform(-3, 3, 300), rng.uniform(0.1, 0.4, 300)], 1)
    sph = np.concatenate([[[0.0, -1e5, 0.0, 1e5]], small])
    n = 100_000
    depth = rng.choice([1e2, 1e3, 1e4, 1e5], n)
    o = np.stack([rng.uniform(-3, 3, n), -depth, rng.uniform(-3, 3, n)], 1)
    target = small[rng.integers(0, len(small), n), :3] + rng.normal(scale=0.2, size=(n, 3))
    _compare(sph, o, target - o)


def test_renders_cull_equals_no_cull(oracle_mod, final_scene):
    cam = P.camera_look_at(aspect=160 / 90)
    a, ra, sa = P.render(final_scene, cam, 160, 90, 8, cull=True, cull_stats=True)
    b, rb, sb = P.render(final_scene, cam, 160, 90, 8, cull=False, cull_stats=True)
    assert np.array_equal(bits(a), bits(b)) and np.array_equal(ra, rb)
    assert sa["rays"] == sb["rays"]
    assert sa["tests_executed"] < sb["tests_executed"] / 5, (sa, sb)
    # the default (non-counting) kernel: same bits and rays, no test counts
    c, rc, sc = P.render(final_scene, cam, 160, 90, 8)
    assert np.array_equal(bits(a), bits(c)) and np.array_equal(ra, rc)
    assert (sc["rays"], sc["rays_traced"]) == (sa["rays"], sa["rays_traced"])
    assert sc["tests_executed"] == 0 and sc["box_tests"] == 0, sc
    want, _, rays = oracle_mod.render(final_scene, cam, 160, 90, 8, threads=8)
    assert np.array_equal(bits(a), bits(want)) and sa["rays"] == rays


def test_renders_of_culled_scenes_vs_oracle(oracle_mod):
    rng = np.random.default_rng(9)
    base = np.concatenate([rng.uniform(-2, 2, (200, 3)), rng.uniform(0.05, 0.4, (200, 1))], 1)
    base[:, 2] -= 4
    for sph in (np.concatenate([base, base]), np.concatenate([[[0, -100.5, 0, 100.0]], base])):
        cam = oracle_mod.camera_default()
        got, _, st = P.render(sph, cam, 48, 27, 3)
        want, _, rays = oracle_mod.render(sph, cam, 48, 27, 3, threads=8)
        assert np.array_equal(bits(got), bits(want))
        assert st["rays"] == rays


def test_trapped_termination_is_bit_identical(oracle_mod, final_scene):
    """ending paths stuck at an exact C == 0 fixed point changes no
    bit and no ray count; it removes most executed work on the final scene."""
    cam = P.camera_look_at(aspect=160 / 90)
    a, ra, sa = P.render(final_scene, cam, 160, 90, 8, fixpoint=True, cull_stats=True)
    b, rb, sb = P.render(final_scene, cam, 160, 90, 8, fixpoint=False, cull_stats=True)
    assert np.array_equal(bits(a), bits(b)) and np.array_equal(ra, rb)
    assert sa["rays"] == sb["rays"]
    assert sa["tests_executed"] < sb["tests_executed"] / 2, (sa, sb)
    assert sb["rays_traced"] == sb["rays"] and sa["rays_traced"] < sa["rays"] / 3, (sa, sb)
    # the counting variant's tallies by kind (bench.py's roofline): FP32
    # pre-rejects, FP32 slab tests and FP64 root-box tests all occur on C3's scene
    assert sa["prerejects"] > 0 and sa["box_tests"] > 0 and sa["root_box_tests"] > 0, sa
    want, _, rays = oracle_mod.render(final_scene, cam, 160, 90, 8, threads=8)
    assert np.array_equal(bits(a), bits(want)) and sa["rays"] == rays


def _contact_scene(rng):
    """Spheres on exact, representable positions: touching pairs, spheres
    resting on a big ground sphere, duplicates, nested and coincident ones —
    the places where an origin can sit on two surfaces at once."""
    s = [[0.0, -1000.0, 0.0, 1000.0]]
    for i in range(-4, 5):
        for k in range(-3, 1):
            r = float(rng.choice([0.25, 0.5, 0.125]))
            s.append([i * 1.0, r, k * 1.0 - 2.0, r])          # resting on y = 0
    s += [[0.0, 1.0, -3.0, 0.5], [1.0, 1.0, -3.0, 0.5]]     # touching pair
    s += [[-1.0, 1.0, -3.0, 0.5], [-1.0, 1.0, -3.0, 0.5]]   # duplicates
    s += [[2.0, 1.0, -3.0, 0.5], [2.0, 1.0, -3.0, 0.25]]    # nested
    s += [[0.5, 2.0, -3.0, 0.5], [0.5, 2.0, -3.0, -0.5]]    # negative radius twin
    return np.array(s)


@pytest.mark.parametrize("seed", [1, 2])
def test_trapped_termination_contact_scenes(oracle_mod, seed):
    sph = _contact_scene(np.random.default_rng(seed))
    cam = P.camera_look_at((0.0, 2.0, 4.0), (0.0, 0.5, -2.0), vfov=50.0, aspect=64 / 40)
    a, ra, sa = P.render(sph, cam, 64, 40, 6, seed=seed, fixpoint=True)
    b, rb, sb = P.render(sph, cam, 64, 40, 6, seed=seed, fixpoint=False)
    assert np.array_equal(bits(a), bits(b)) and np.array_equal(ra, rb)
    assert sa["rays"] == sb["rays"]
    want, _, rays = oracle_mod.render(sph, cam, 64, 40, 6, seed=seed, threads=8)
    assert np.array_equal(bits(a), bits(want)) and sa["rays"] == rays


def test_camera_lists_are_bit_identical(oracle_mod, final_scene, knobs):
    """camera rays tested against per-pixel candidate lists give
    the same frame as the BVH walk, for the benchmark camera and for cameras
    close to / inside spheres, wide and narrow fields, and a 1:3 shard."""
    cams = [P.camera_look_at(aspect=96 / 64),
            P.camera_look_at((4.0, 1.0, 0.5), (4.0, 1.0, -3.0), vfov=90.0, aspect=96 / 64),
            P.camera_look_at((-4.0, 1.2, 0.0), (0.0, 0.2, 0.0), vfov=120.0, aspect=96 / 64),
            P.camera_look_at((0.0, 0.3, 2.0), (0.0, 0.2, -5.0), vfov=5.0, aspect=96 / 64)]
    for cam in cams:
        for off, stride in ((0, 1), (1, 3)):
            a, _, sa = P.render(final_scene, cam, 96, 64, 3, row_offset=off, row_stride=stride)
            knobs("no_camlist", 1)
            b, _, sb = P.render(final_scene, cam, 96, 64, 3, row_offset=off, row_stride=stride)
            knobs("no_camlist", 0)
            assert np.array_equal(bits(a), bits(b)) and sa["rays"] == sb["rays"]
            want, _, rays = oracle_mod.render(final_scene, cam, 96, 64, 3, row_offset=off,
                                              row_stride=stride, threads=8)
            assert np.array_equal(bits(a), bits(want)) and sa["rays"] == rays


def test_neighbour_lists_are_bit_identical(oracle_mod, final_scene, knobs):
    """rays that re-hit their start sphere test only its
    neighbours; the frames equal the grid/BVH path's and the oracle's, on the
    final scene and on contact scenes (touching, duplicate, nested spheres)."""
    scenes = [(final_scene, P.camera_look_at(aspect=96 / 64))]
    for seed in (1, 2):
        scenes.append((_contact_scene(np.random.default_rng(seed)),
                       P.camera_look_at((0.0, 2.0, 4.0), (0.0, 0.5, -2.0), vfov=50.0,
                                        aspect=96 / 64)))
    for sph, cam in scenes:
        a, _, sa = P.render(sph, cam, 96, 64, 4)
        knobs("no_neighbors", 1)
        b, _, sb = P.render(sph, cam, 96, 64, 4)
        knobs("no_neighbors", 0)
        assert np.array_equal(bits(a), bits(b)) and sa["rays"] == sb["rays"]
        want, _, rays = oracle_mod.render(sph, cam, 96, 64, 4, threads=8)
        assert np.array_equal(bits(a), bits(want)) and sa["rays"] == rays


def test_far_camera_rebase_bit_exact(oracle_mod, final_scene):
    """A camera 2^34 (1.7e10) units out on the z axis, looking back at the
    scene through a 2e-8 degree field (about 6 units high there). Its rays'
    root-box entry, kept as a float, would move a re-based origin far outside
    the range the FP32 slab test's error bound covers, and the
    reference's own FP64 sphere test no longer resolves unit spheres there
    (its roots err by hundreds of units): such origins (beyond 8 r_check)
    take the linear scan, and the frame, noise as it is, equals the oracle's
    bit for bit. (On the z axis the camera's x / y direction components stay
    exact.)"""
    cam = P.camera_look_at((0.0, 0.5, 2.0 ** 34), (0.0, 0.5, 0.0), vfov=2e-8, aspect=48 / 32)
    a, _, sa = P.render(final_scene, cam, 48, 32, 3, seed=5, cull_stats=True)
    want, _, rays = oracle_mod.render(final_scene, cam, 48, 32, 3, seed=5, threads=8)
    assert np.array_equal(bits(a), bits(want)) and sa["rays"] == rays
    assert sa["tests_executed"] >= 48 * 32 * 3 * 484, sa  # camera rays: the linear scan
    # Ray by ray (the hittable_list::hit probe shares hit_quick and the
    # walk): origins 2^9 .. 2^36 out, aimed at the scene without its ground
    # (so nothing ends them before the walk), against the reference scan.
    # Up to 8 r_check (~6200 units here) they take the FP64 root-box test and
    # the re-based walk; beyond it the reference's own roots may err by more
    # than the BVH pad (they do, by hundreds of units at 2^30), so those rays
    # take the linear scan.
    rng = np.random.default_rng(41)
    n = 300_000
    small = final_scene[1:]
    o = rng.normal(size=(n, 3))
    o *= (2.0 ** rng.uniform(9, 36, (n, 1))) / np.linalg.norm(o, axis=1, keepdims=True)
    d = np.concatenate([rng.uniform(-12, 12, (n, 1)), rng.uniform(0, 2, (n, 1)),
                        rng.uniform(-12, 12, (n, 1))], 1) - o
    _compare(small, o, d)


def test_enclosing_sky_sphere(oracle_mod, final_scene):
    """a non-BVH sphere around the final scene, of radius 1e6 (the
    largest coordinate the culling structure accepts; beyond it the whole scene
    takes the linear scan). Every ray that leaves the scene hits it from inside
    and scatters back from ~1e6 out, beyond 8 r_check: those rays take the
    reference's scan while the scene's rays keep the culled
    paths. Frame and ray count equal the oracle's, and probe rays from the sky
    sphere's surface into the scene equal the linear sweep."""
    sph = np.concatenate([final_scene, [[0.0, 0.0, 0.0, 1e6]]])
    cam = P.camera_look_at(aspect=48 / 32)
    a, _, sa = P.render(sph, cam, 48, 32, 2, seed=7, cull_stats=True)
    want, _, rays = oracle_mod.render(sph, cam, 48, 32, 2, seed=7, threads=8)
    assert np.array_equal(bits(a), bits(want)) and sa["rays"] == rays
    assert sa["box_tests"] > 0 and sa["tests_executed"] > 100 * len(sph), sa
    rng = np.random.default_rng(43)
    n = 50_000
    u = rng.normal(size=(n, 3))
    o = 1e6 * u / np.linalg.norm(u, axis=1, keepdims=True)
    d = final_scene[rng.integers(1, len(final_scene), n), :3] + rng.normal(scale=0.3, size=(n, 3)) - o
    _compare(sph, o, d)


def test_grazing_bounce_rays_near_neighbours(final_scene):
    """Hinted bounce rays that graze the spheres nearest their start sphere j
    (the neighbour-list and BVH-leaf culling's hardest case; the escape-table
    experiment of r05, profiles/r05_escape, was checked with them): rays from
    j's surface (within the pad/4 band) aimed at the silhouettes of j's 8
    nearest spheres (tangent +- 1e-12 .. 1e-4), against the reference scan."""
    rng = np.random.default_rng(91)
    sph = final_scene
    bvh = np.where(np.abs(sph[:, 3]) < 16 * np.median(np.abs(sph[:, 3])))[0]
    c = sph[:, :3]
    n = 300_000
    dist = np.linalg.norm(c[bvh][None, :, :] - c[bvh][:, None, :], axis=2)  # BVH x BVH
    np.fill_diagonal(dist, np.inf)
    near8 = bvh[np.argsort(dist, axis=1)[:, :8]]  # the 8 nearest to each BVH sphere
    jj = rng.integers(0, len(bvh), n)
    j = bvh[jj]
    k = near8[jj, rng.integers(0, 8, n)]
    u = rng.normal(size=(n, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    rj = np.abs(sph[j, 3])
    o = c[j] + (rj * (1 + rng.choice([0.0, 1e-15, -1e-15, 3e-6, -3e-6], n)))[:, None] * u
    w = c[k] - o
    w /= np.linalg.norm(w, axis=1, keepdims=True)
    perp = rng.normal(size=(n, 3))
    perp -= (perp * w).sum(1, keepdims=True) * w
    perp /= np.linalg.norm(perp, axis=1, keepdims=True)
    eps = rng.choice([0.0, 1e-12, -1e-12, 1e-7, -1e-7, 1e-4, 3e-4], n)
    d = (c[k] + (np.abs(sph[k, 3]) * (1 + eps))[:, None] * perp) - o
    _compare_hinted(sph, o, d, j)
