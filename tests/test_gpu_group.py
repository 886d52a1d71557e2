"""The native multi-device path (rt_group, include/rt.h; psrt_group.cpp):
one frame over G members, each with its own context and host thread,
interleaved rows gathered into reference pixel order in host memory
(the reference loop main.cc:72-88). The pool's boxes have
one GPU, so the members share it: G = 2, 3, 8 members must give the
one-device frame bit for bit, and the C4 rows the reference rendered."""
import hashlib
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, bits, golden, unhex

import petershirleyraytracer_amd as P

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("G", [2, 3, 8])
def test_group_equals_one_device_c3_scene(final_scene, G):
    """The C3 workload's scene and camera at 96 x 64 x 100 spp."""
    w, h, spp = 96, 64, 100
    cam = P.camera_look_at(aspect=1.5)
    want, wrgb, ws = P.render(final_scene, cam, w, h, spp, seed=3)
    g = P.DeviceGroup([0] * G)
    try:
        g.set_scene(final_scene, cam)
        got, rgb, st = g.render(w, h, spp, seed=3)
        assert np.array_equal(bits(got), bits(want)) and np.array_equal(rgb, wrgb)
        assert (st["rays"], st["samples"], st["rays_traced"]) == (ws["rays"], ws["samples"],
                                                                  ws["rays_traced"])
        # a shard of the frame over the group: the group splits the shard's rows
        s_acc, _, _ = g.render(w, h, spp, seed=3, row_offset=1, row_stride=3)
        assert np.array_equal(bits(s_acc), bits(want[1::3]))
    finally:
        g.close()


def test_group_c4_rows_match_reference_pixels(final_scene):
    """C4 (3840 x 2160 x 500, the BASELINE's 8-GPU frame): 8 rows through
    8 members (one row each), against the pixels the reference rendered and
    against one device."""
    fx = golden("counter_final.json")
    grp = next(s for s in fx["sampled"] if s["width"] == 3840)
    w, h, spp = grp["width"], grp["height"], grp["spp"]
    cam = np.array(unhex(grp["camera"]))
    p0 = grp["pixels"][0]
    stride = h // 8  # 270: 8 rows, one per member, p0's row among them
    off = p0["row"] % stride
    g = P.DeviceGroup([0] * 8)
    try:
        g.set_scene(final_scene, cam)
        acc, _, st = g.render(w, h, spp, grp["max_depth"], grp["seed"], off, stride)
    finally:
        g.close()
    assert acc.shape == (8, w, 3)
    for p in grp["pixels"]:
        if p["row"] % stride == off:
            k = (p["row"] - off) // stride
            assert np.array_equal(bits(acc[k, p["i"]]), bits(unhex(p["accum"]))), p
    one, _, so = P.render(final_scene, cam, w, h, spp, grp["max_depth"], grp["seed"],
                          row_offset=off, row_stride=stride)
    assert np.array_equal(bits(acc), bits(one)) and st["rays"] == so["rays"]


def test_render_devices_one_shot_and_more_members_than_rows(oracle_mod):
    two = P.scene_two_spheres()
    cam = P.camera_default()
    want, wrgb, _ = oracle_mod.render(two, cam, 40, 6, 4, threads=8)
    # 8 members for 6 rows: two members own none
    got, rgb, st = P.render_devices(two, cam, 40, 6, 4, [0] * 8)
    assert np.array_equal(bits(got), bits(want)) and np.array_equal(rgb, wrgb)
    assert st["samples"] == 40 * 6 * 4


def test_cli_devices(tmp_path):
    """bin/raytracer --devices: the reference main() over a device group
    (include/psrt/render.hpp psrt::render(..., devices)); same P3 bytes and
    accumulators as one device and as the reference's 120 x 80 x 8 frame."""
    exe = os.path.join(ROOT, "petershirleyraytracer_amd", "bin", "raytracer")
    outs = {}
    for tag, extra in (("one", []), ("three", ["--devices", "0,0,0"]), ("n1", ["--devices", "1"])):
        out, acc = tmp_path / f"{tag}.ppm", tmp_path / f"{tag}.bin"
        subprocess.run([exe, "--scene", "final", "--width", "120", "--height", "80", "--spp", "8",
                        "-o", str(out), "--accum", str(acc), *extra], check=True, timeout=120)
        outs[tag] = (hashlib.md5(out.read_bytes()).hexdigest(),
                     hashlib.sha256(acc.read_bytes()).hexdigest())
    assert outs["one"] == outs["three"] == outs["n1"]
    want = golden("counter_final.json")["cases"][1]  # the reference's 120 x 80 x 8 frame
    assert (want["width"], want["height"], want["spp"]) == (120, 80, 8)
    assert outs["three"] == (want["p3_md5"], want["accum_sha256"])


def test_group_render_checks_params_first():
    """rt_group_render runs rt_render's parameter check before any member's
    shard arithmetic or buffer sizing: a negative width is
    RT_E_INVALID (not RT_E_NOMEM from a huge allocation), and a row stride whose
    product with the member count overflows int is rejected."""
    import ctypes as C
    from petershirleyraytracer_amd import _lib
    L = _lib.load()
    g = P.DeviceGroup([0, 0])
    g.set_scene(P.scene_two_spheres(), P.camera_default())
    acc = (C.c_double * 48)()
    for kw in (dict(width=-5, height=4), dict(width=4, height=4, row_stride=2 ** 30 + 1),
               dict(width=4, height=4, spp=0)):
        args = dict(width=4, height=4, spp=1)
        args.update(kw)
        p = P.params(args["width"], args["height"], args["spp"],
                     row_stride=args.get("row_stride", 1))
        assert L.rt_group_render(g.handle, C.byref(p), acc, None, None) == -1, kw
    g.close()
