"""Culling known answers from the REFERENCE ITSELF.

The device's exact culling (BVH, grid and 2x2x2 block lists, neighbour lists,
pre-rejects) must return the record of the reference's
linear scan, hittable_list::hit (hittable_list.cc:3-20) over sphere::hit
(sphere.cc:3-40). tests/test_gpu_culling.py checks that against the device's
own linear sweep on millions of rays; this fixture anchors a set of the same
adversarial rays directly on the reference: oracle/_ref/ref_render
--kat-scene (the reference sources compiled unmodified) answers every ray,
and tests/test_gpu_culling_kat.py compares the device's CULLED record with it
bit for bit.

Ray families (per scene): origins on sphere surfaces (exact and a few ulp /
~pad off) with scatter, uniform and silhouette-grazing directions, the
previous-hit sphere as the hint; grazing rays at +-1e-15..1e-6 of tangency;
random interior points; far origins (50-3000 units, inside the r=1000
ground); camera rays; short segments crossing grid cells. Scenes: the final
scene, duplicated, touching, nested, mixed big / tiny, tall, negative-radius,
coincident, sparse and contact scenes, and a 1e5 ground with origins deep
inside it.

    python tests/golden/make_culling_kat.py     # ~1 min; writes culling_kat.npz
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import oracle as O  # noqa: E402


def on_surface(sph, idx, rng, mode):
    n = len(idx)
    c, r = sph[idx, :3], np.abs(sph[idx, 3])
    u = rng.normal(size=(n, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    scale = max(1.0, float(np.max(np.abs(sph[:, :3]) + np.abs(sph[:, 3:4]))))
    off = rng.choice([0.0, 0.0, 1e-16, -1e-16, 1e-12, -1e-12, 2e-5 * scale / 64,
                      -2e-5 * scale / 64], n)
    o = c + (r * (1 + off))[:, None] * u
    if mode == "scatter":  # n + random_in_hemisphere(n) (vec3.h:102-109, main.cc:42)
        v = rng.uniform(-1, 1, (n, 3))
        v /= np.maximum(1.0, np.linalg.norm(v, axis=1, keepdims=True))
        v = np.where(((v * u).sum(1) > 0)[:, None], v, -v)
        return o, u + v
    if mode == "inward":  # scatter about the flipped normal (back-face hits)
        v = rng.uniform(-1, 1, (n, 3))
        v /= np.maximum(1.0, np.linalg.norm(v, axis=1, keepdims=True))
        v = np.where(((v * -u).sum(1) > 0)[:, None], v, -v)
        return o, -u + v
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


def tangent(sph, n, rng):
    idx = rng.integers(0, len(sph), n)
    c, r = sph[idx, :3], np.abs(sph[idx, 3])
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    perp = rng.normal(size=(n, 3))
    perp -= (perp * d).sum(1, keepdims=True) * d
    perp /= np.linalg.norm(perp, axis=1, keepdims=True)
    eps = rng.choice([0.0, 1e-15, -1e-15, 1e-9, -1e-9, 1e-6], n)
    p = c + (r * (1 + eps))[:, None] * perp
    o = p - rng.uniform(0.0, 30.0, n)[:, None] * d
    return o, d * rng.uniform(0.1, 3.0, (n, 1))


def ray_set(sph, n, rng, final=False):
    """(o, d, hint) for one scene: ~n rays over the families above."""
    parts = []
    m = n // 8
    for mode in ("scatter", "inward", "uniform", "silhouette"):
        idx = rng.integers(0, len(sph), m)
        if final:
            idx[: m // 3] = 0  # the ground (a big sphere), on points near the field
        o, d = on_surface(sph, idx, rng, mode)
        if final and mode in ("scatter", "uniform"):
            g = idx == 0
            pg = np.stack([rng.uniform(-13, 13, g.sum()), np.zeros(g.sum()),
                           rng.uniform(-13, 13, g.sum())], 1)
            pg[:, 1] = -1000.0 + np.sqrt(1000.0 ** 2 - pg[:, 0] ** 2 - pg[:, 2] ** 2)
            o[g] = pg
            if mode == "scatter":
                ng = (pg - [0.0, -1000.0, 0.0]) / 1000.0
                v = rng.uniform(-1, 1, (g.sum(), 3))
                v /= np.maximum(1.0, np.linalg.norm(v, axis=1, keepdims=True))
                v = np.where(((v * ng).sum(1) > 0)[:, None], v, -v)
                d[g] = ng + v
        parts.append((o, d, idx.astype(np.int32)))
    o, d = tangent(sph, m, rng)
    parts.append((o, d, np.full(m, -1, np.int32)))
    lo = sph[:, :3].min(0) - 2.0
    hi = sph[:, :3].max(0) + 2.0
    o = rng.uniform(lo, hi, (m, 3))
    parts.append((o, rng.normal(size=(m, 3)), np.full(m, -1, np.int32)))
    o = rng.normal(size=(m, 3)) * rng.choice([50.0, 500.0, 3000.0], (m, 1))
    parts.append((o, rng.uniform(lo, hi, (m, 3)) - o, np.full(m, -1, np.int32)))
    if final:  # short segments down to the ground among the small spheres
        o = np.stack([rng.uniform(-12, 12, m), rng.uniform(1e-4, 0.6, m), rng.uniform(-12, 12, m)], 1)
        reach, ang = rng.uniform(0.02, 2.0, m), rng.uniform(0, 2 * np.pi, m)
        d = np.stack([reach * np.cos(ang), -o[:, 1], reach * np.sin(ang)], 1)
        parts.append((o, d * rng.uniform(0.5, 2.0, (m, 1)), np.full(m, -1, np.int32)))
    else:
        o, d = tangent(sph, m, rng)
        parts.append((o, d, np.full(m, -1, np.int32)))
    o = np.concatenate([p[0] for p in parts])
    d = np.concatenate([p[1] for p in parts])
    h = np.concatenate([p[2] for p in parts])
    return np.ascontiguousarray(np.concatenate([o, d], 1)), h


def scenes(rng):
    base = np.concatenate([rng.uniform(-3, 3, (300, 3)), rng.uniform(0.05, 0.6, (300, 1))], 1)
    contact = [[0.0, -1000.0, 0.0, 1000.0]]
    for i in range(-4, 5):
        for k in range(-3, 1):
            r = float(rng.choice([0.25, 0.5, 0.125]))
            contact.append([i * 1.0, r, k * 1.0 - 2.0, r])
    contact += [[0.0, 1.0, -3.0, 0.5], [1.0, 1.0, -3.0, 0.5], [-1.0, 1.0, -3.0, 0.5],
                [-1.0, 1.0, -3.0, 0.5], [2.0, 1.0, -3.0, 0.5], [2.0, 1.0, -3.0, 0.25],
                [0.5, 2.0, -3.0, 0.5], [0.5, 2.0, -3.0, -0.5]]
    small = np.stack([rng.uniform(-3, 3, 300), rng.uniform(-0.2, 0.2, 300),
                      rng.uniform(-3, 3, 300), rng.uniform(0.1, 0.4, 300)], 1)
    return {
        "duplicates": np.concatenate([base, base[::-1]]),
        "touching": np.array([[x, 0.0, z, 0.5] for x in range(-6, 7) for z in range(-6, 7)],
                             dtype=np.float64),
        "nested": np.concatenate([base, base * [1, 1, 1, 0.5], base * [1, 1, 1, 0.25]]),
        "mixed_big": np.concatenate([base, [[0, -1000, 0, 1000], [0, 0, 0, 40.0],
                                            [5, 5, 5, 1e-9]]]),
        "tall": np.concatenate([base, np.concatenate([rng.uniform(-3, 3, (12, 3)),
                                                      rng.uniform(1.2, 4.0, (12, 1))], 1)]),
        "negative_r": base * [1, 1, 1, -1],
        "coincident": np.tile([[0.0, 0.0, 0.0, 1.0]], (40, 1)),
        "sparse": np.concatenate([rng.uniform(-40, 40, (60, 3)), rng.uniform(0.2, 1.0, (60, 1))], 1),
        "contact": np.array(contact),
        "huge_ground": np.concatenate([[[0.0, -1e5, 0.0, 1e5]], small]),
    }


def reference_answers(sph, rays, procs=8):
    """ref_render --kat-scene over the rays (split over `procs` processes).
    Returns records [N, 9] = (index, p, normal, t, front_face), index -1 = miss."""
    chunks = np.array_split(np.arange(len(rays)), procs)
    head = " ".join([str(len(sph))] + [float(v).hex() for s in sph for v in s]) + "\n"

    def one(ix):
        with tempfile.TemporaryDirectory() as td:
            p = os.path.join(td, "k.txt")
            with open(p, "w") as f:
                f.write(head)
                for k in ix:
                    f.write(" ".join(float(v).hex() for v in rays[k]) + " 0x0p+0 inf\n")
            out = subprocess.run([O.REF_BIN, "--kat-scene", p], check=True,
                                 capture_output=True).stdout.decode().split("\n")
        rec = np.zeros((len(ix), 9))
        for row, line in enumerate(out[:len(ix)]):
            t = line.split()
            rec[row, 0] = int(t[0])
            if int(t[0]) >= 0:
                rec[row, 1:8] = [float.fromhex(v) for v in t[1:8]]
                rec[row, 8] = float(int(t[8]))
        return rec

    with ThreadPoolExecutor(procs) as ex:
        return np.concatenate(list(ex.map(one, chunks)))


def main():
    assert O.have_ref(), "build oracle/_ref/ref_render first: make -C oracle"
    rng = np.random.default_rng(20250303)
    out = {}
    sets = [("final", O.scene_random_spheres(1), 16000, True)]
    sets += [(name, sph, 3200, False) for name, sph in scenes(rng).items()]
    total = 0
    for name, sph, n, final in sets:
        sph = np.ascontiguousarray(sph, dtype=np.float64)
        rays, hints = ray_set(sph, n, rng, final)
        if name == "final":  # camera rays of the bench configuration
            cam = O.camera_look_at(aspect=1.5)
            u, v = rng.uniform(0, 1, 2000), rng.uniform(0, 1, 2000)
            d = cam[1] + u[:, None] * cam[2] + v[:, None] * cam[3] - cam[0]
            cr = np.concatenate([np.broadcast_to(cam[0], (2000, 3)), d], 1)
            rays = np.concatenate([rays, cr])
            hints = np.concatenate([hints, np.full(2000, -1, np.int32)])
        if name == "huge_ground":  # origins deep inside the ground, aimed at the sunk spheres
            m = 2000
            small = sph[1:]
            depth = rng.choice([1e2, 1e3, 1e4, 1e5], m)
            o = np.stack([rng.uniform(-3, 3, m), -depth, rng.uniform(-3, 3, m)], 1)
            tgt = small[rng.integers(0, len(small), m), :3] + rng.normal(scale=0.2, size=(m, 3))
            rays = np.concatenate([rays, np.concatenate([o, tgt - o], 1)])
            hints = np.concatenate([hints, np.full(m, -1, np.int32)])
        rec = reference_answers(sph, rays)
        out[f"{name}__spheres"] = sph
        out[f"{name}__rays"] = rays
        out[f"{name}__hints"] = hints.astype(np.int32)
        out[f"{name}__index"] = rec[:, 0].astype(np.int32)
        out[f"{name}__t"] = rec[:, 7]
        # the full records (index, p, normal, t, front_face) as bytes, hashed:
        # the device's must hash the same
        out[f"{name}__sha256"] = np.frombuffer(
            hashlib.sha256(np.ascontiguousarray(rec).tobytes()).digest(), dtype=np.uint8)
        total += len(rays)
        print(name, len(sph), "spheres", len(rays), "rays", f"hit rate {(rec[:, 0] >= 0).mean():.3f}",
              flush=True)
    np.savez(os.path.join(HERE, "culling_kat.npz"), **out)
    print("total rays", total)


if __name__ == "__main__":
    main()
