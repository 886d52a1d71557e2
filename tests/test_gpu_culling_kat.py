"""The device's CULLED hittable_list::hit against the reference itself.

tests/golden/culling_kat.npz (tests/golden/make_culling_kat.py) holds 52k
adversarial rays over the final scene and ten contact / degenerate scenes,
answered by the reference sources compiled unmodified (oracle/_ref/ref_render
--kat-scene: hittable_list.cc:3-20 over sphere.cc:3-40). The device runs
them through its exact-culling path (BVH walk, grid and block lists,
neighbour lists behind the previous-hit hint, camera rays, pre-rejects,
far-origin root-box test) via rt_debug_world_hit_hint; every record (index,
p, normal, t, front_face) must equal the reference's bit for bit.
"""
import hashlib
import os

import numpy as np
import pytest

from conftest import ROOT, bits

FIX = os.path.join(ROOT, "tests", "golden", "culling_kat.npz")


def _scenes():
    z = np.load(FIX, allow_pickle=False)
    names = sorted({k.split("__")[0] for k in z.files})
    return z, names


def test_fixture_is_pinned_by_the_oracle_restatement(oracle_mod):
    """CPU: the oracle's world_hit (rt_oracle.c) gives the reference's answers."""
    z, names = _scenes()
    for name in names:
        sph, rays = z[f"{name}__spheres"], z[f"{name}__rays"]
        idx, t = z[f"{name}__index"], z[f"{name}__t"]
        sel = np.linspace(0, len(rays) - 1, min(len(rays), 400)).astype(int)
        for k in sel:
            i, rec = oracle_mod.world_hit(sph, rays[k, :3], rays[k, 3:], 0.0, np.inf)
            assert i == idx[k], (name, k, i, idx[k])
            if i >= 0:
                assert bits(np.float64(rec[6])) == bits(np.float64(t[k])), (name, k)


@pytest.mark.gpu
def test_culled_records_equal_the_reference():
    from petershirleyraytracer_amd.render import world_hit
    z, names = _scenes()
    total = 0
    for name in names:
        sph, rays, hints = z[f"{name}__spheres"], z[f"{name}__rays"], z[f"{name}__hints"]
        r8 = np.concatenate([rays, np.zeros((len(rays), 1)), np.full((len(rays), 1), np.inf)], 1)
        got = world_hit(sph, r8, cull=True, hints=hints)
        gi = got[:, 0].astype(np.int32)
        bad = np.where(gi != z[f"{name}__index"])[0]
        assert len(bad) == 0, (name, len(bad), bad[:5], gi[bad[:5]], z[f"{name}__index"][bad[:5]])
        assert np.array_equal(bits(got[:, 7]), bits(z[f"{name}__t"])), name
        digest = hashlib.sha256(np.ascontiguousarray(got).tobytes()).digest()
        assert digest == bytes(z[f"{name}__sha256"]), name  # p, normal, front_face too
        # the same rays without the hint (camera-ray / grid / walk paths)
        got2 = world_hit(sph, r8, cull=True)
        assert hashlib.sha256(np.ascontiguousarray(got2).tobytes()).digest() == \
            bytes(z[f"{name}__sha256"]), name
        total += len(rays)
    assert total >= 50_000
