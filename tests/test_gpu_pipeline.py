"""Frames in flight (DESIGN.md §7 "Frame pipelining"): contexts rendering at
the same time on their own streams, and the per-context camera-list cache
(§4 psrt_camera_lists), must give the same bits as one render at a time."""
import numpy as np
import pytest

import petershirleyraytracer_amd as P

pytestmark = pytest.mark.gpu

W, H, SPP = 96, 64, 8


def _serial(sph, cam, **kw):
    acc, rgb, _ = P.render(sph, cam, W, H, SPP, **kw)
    return acc, rgb


def _device_buffers(rows, n=1):
    import torch
    acc = [torch.zeros((rows, W, 3), dtype=torch.float64, device="cuda:0") for _ in range(n)]
    rgb = [torch.zeros((rows, W, 3), dtype=torch.uint8, device="cuda:0") for _ in range(n)]
    return acc, rgb


def test_contexts_in_flight_on_their_own_streams():
    import torch
    sph = P.scene_random_spheres(1)
    cam = P.camera_look_at(aspect=W / H)
    want_acc, want_rgb = _serial(sph, cam)
    ctxs = [P.Context(0) for _ in range(3)]
    for c in ctxs:
        c.set_scene(sph, cam)
    acc, rgb = _device_buffers(H, 3)
    prm = P.params(W, H, SPP)
    for rep in range(2):  # the second round reuses the cached camera lists
        for k, c in enumerate(ctxs):  # all enqueued before any wait
            c.render_device(prm, acc[k].data_ptr(), rgb[k].data_ptr(), c.stream())
        for k, c in enumerate(ctxs):
            st = c.sync_stats()
            assert st["samples"] == W * H * SPP
        torch.cuda.synchronize()
        for k in range(3):
            a = acc[k].cpu().numpy()
            assert np.array_equal(a.view(np.uint64), want_acc.view(np.uint64)), (rep, k)
            assert np.array_equal(rgb[k].cpu().numpy(), want_rgb), (rep, k)


def test_camera_list_cache_follows_shard_and_camera():
    import torch
    sph = P.scene_random_spheres(1)
    ctx = P.Context(0)
    for look in [(13.0, 2.0, 3.0), (0.0, 1.0, 6.0)]:
        cam = P.camera_look_at(lookfrom=look, aspect=W / H)
        ctx.set_scene(sph, cam)  # a new camera must rebuild the lists
        full, _ = _serial(sph, cam)
        for g in (1, 3, 2, 3):  # shard changes, and a repeated shard (cache hit)
            for r in range(g):
                rows = P.rows_owned(H, r, g)
                acc, rgb = _device_buffers(rows)
                ctx.render_device(P.params(W, H, SPP, 50, 0, r, g), acc[0].data_ptr(),
                                  rgb[0].data_ptr(), 0)
                ctx.sync_stats()
                torch.cuda.synchronize()
                # shard rows are reference rows r, r+g, ... counted from the top
                want = full[r::g]
                got = acc[0].cpu().numpy()
                assert np.array_equal(got.view(np.uint64), want.view(np.uint64)), (look, g, r)
