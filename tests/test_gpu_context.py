"""Context and threading contract of the C ABI (include/rt.h), on an MI355X.

- Renders of one rt_context on different streams (a caller's torch streams)
  are ordered by the library: set_scene, a re-shard (camera-list rebuild) or a
  buffer reallocation never touches buffers an in-flight render still reads.
- rt_render is safe to call from several host threads (per-device lock).
- The kernel's 32-bit per-lane counters flush to the 64-bit totals before
  they can wrap (the flush_at tuning knob forces the flush path on every refill block).
- A shard that owns no rows (more ranks than rows) renders nothing.

Expected values come from the oracle restatement (pinned to the reference's
fixtures by tests/test_oracle.py); the bar is bit-identical FP64 accumulators.
"""
import os
import threading

import numpy as np
import pytest

from conftest import bits

import petershirleyraytracer_amd as P

pytestmark = pytest.mark.gpu


def test_renders_on_caller_streams_are_ordered(oracle_mod):
    import torch
    dev = torch.device("cuda", 0)
    fin = oracle_mod.scene_random_spheres(1)
    two = oracle_mod.scene_two_spheres()
    cam_f = oracle_mod.camera_look_at(aspect=160 / 96)
    cam_t = oracle_mod.camera_default()
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    ctx = P.Context(0)
    ctx.set_scene(fin, cam_f)
    # frame A on s1: long enough to still be running when the host moves on
    a = torch.zeros((96, 160, 3), dtype=torch.float64, device=dev)
    ctx.render_device(P.params(160, 96, 64), a.data_ptr(), 0, s1.cuda_stream)
    # new scene while A may run; frame B on s2 (bigger: sample buffer grows)
    ctx.set_scene(two, cam_t)
    b = torch.zeros((108, 192, 3), dtype=torch.float64, device=dev)
    ctx.render_device(P.params(192, 108, 40), b.data_ptr(), 0, s2.cuda_stream)
    # back on s1, another shard of the same scene (camera lists rebuilt)
    c = torch.zeros((54, 192, 3), dtype=torch.float64, device=dev)
    ctx.render_device(P.params(192, 108, 40, row_offset=1, row_stride=2), c.data_ptr(), 0,
                      s1.cuda_stream)
    st = ctx.sync_stats()
    torch.cuda.synchronize(dev)
    want_a, _, _ = oracle_mod.render(fin, cam_f, 160, 96, 64, threads=8)
    want_b, _, rays_b = oracle_mod.render(two, cam_t, 192, 108, 40, threads=8)
    assert np.array_equal(bits(a.cpu().numpy()), bits(want_a))
    assert np.array_equal(bits(b.cpu().numpy()), bits(want_b))
    assert np.array_equal(bits(c.cpu().numpy()), bits(want_b[1::2]))
    assert st["samples"] == 54 * 192 * 40
    # and a final-scene re-render on s2 after all that (scene swapped back)
    ctx.set_scene(fin, cam_f)
    ctx.render_device(P.params(160, 96, 64), a.data_ptr(), 0, s2.cuda_stream)
    ctx.sync_stats()
    torch.cuda.synchronize(dev)
    assert np.array_equal(bits(a.cpu().numpy()), bits(want_a))
    ctx.close()


def test_rt_render_from_threads(oracle_mod):
    """ctypes drops the GIL: the calls really overlap on the host."""
    fin = oracle_mod.scene_random_spheres(1)
    two = oracle_mod.scene_two_spheres()
    jobs = [(fin, oracle_mod.camera_look_at(aspect=96 / 48), 96, 48, 6),
            (two, oracle_mod.camera_default(), 128, 72, 9),
            (fin, oracle_mod.camera_look_at(aspect=64 / 64), 64, 64, 5)]
    want = [oracle_mod.render(s, c, w, h, n, threads=8)[0] for s, c, w, h, n in jobs]
    errors = []

    def worker(t):
        try:
            for it in range(6):
                k = (t + it) % len(jobs)
                s, c, w, h, n = jobs[k]
                got, _, _ = P.render(s, c, w, h, n)
                if not np.array_equal(bits(got), bits(want[k])):
                    errors.append((t, it, k))
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errors, errors


@pytest.mark.parametrize("flush_at", ["1", "7"])
def test_counter_flush_keeps_totals(oracle_mod, knobs, flush_at):
    """rays / tests stay exact when the per-lane counters flush mid-launch,
    also at max_depth 100000 (trapped paths add max_depth - k at once)."""
    two = oracle_mod.scene_two_spheres()
    cam = oracle_mod.camera_default()
    fin = oracle_mod.scene_random_spheres(1)
    cam_f = oracle_mod.camera_look_at(aspect=48 / 32)
    base = {}
    for key, (s, c, w, h, n, d) in {"two": (two, cam, 40, 20, 3, 100000),
                                     "fin": (fin, cam_f, 48, 32, 4, 50)}.items():
        knobs("flush_at", 0)
        acc0, _, st0 = P.render(s, c, w, h, n, d, cull_stats=True)
        knobs("flush_at", int(flush_at))
        acc1, _, st1 = P.render(s, c, w, h, n, d, cull_stats=True)
        assert np.array_equal(bits(acc0), bits(acc1)), key
        for f in ("rays", "tests_executed", "box_tests", "rays_traced"):
            assert st0[f] == st1[f], (key, f)
        base[key] = (acc1, st1)
    want, _, rays = oracle_mod.render(two, cam, 40, 20, 3, 100000, threads=8)
    assert np.array_equal(bits(base["two"][0]), bits(want))
    assert base["two"][1]["rays"] == rays
    assert rays > 2 ** 24  # trapped paths at depth 1e5 dominate the count


def test_empty_shard(oracle_mod):
    import torch
    two = oracle_mod.scene_two_spheres()
    cam = oracle_mod.camera_default()
    acc, rgb, st = P.render(two, cam, 16, 3, 2, row_offset=5, row_stride=8)
    assert acc.shape == (0, 16, 3) and rgb.shape == (0, 16, 3)
    assert st["samples"] == 0 and st["rays"] == 0
    ctx = P.Context(0)
    ctx.set_scene(two, cam)
    ctx.render_device(P.params(16, 3, 2, row_offset=3, row_stride=4))
    st = ctx.sync_stats()
    assert st["samples"] == 0
    # the context still renders normally afterwards
    out = torch.zeros((3, 16, 3), dtype=torch.float64, device="cuda:0")
    ctx.render_device(P.params(16, 3, 2), out.data_ptr())
    ctx.sync_stats()
    want, _, _ = oracle_mod.render(two, cam, 16, 3, 2)
    assert np.array_equal(bits(out.cpu().numpy()), bits(want))
    ctx.close()


def test_render_into_pinned_host_memory():
    """write_color's bytes may go straight to pinned host memory (bench.py's
    timed step: psrt_reduce's 16-B stores across the link are the frame's
    device-to-host transfer): same bytes as a device buffer, for a frame whose
    row width makes the last wave partial and the 16-B path both taken."""
    import torch
    sph = P.scene_random_spheres(1)
    for (w, h) in ((96, 64), (37, 11)):
        cam = P.camera_look_at(aspect=w / h)
        ctx = P.Context(0)
        ctx.set_scene(sph, cam)
        dev = torch.zeros((h, w, 3), dtype=torch.uint8, device="cuda:0")
        host = torch.zeros((h, w, 3), dtype=torch.uint8, pin_memory=True)
        acc = torch.zeros((h, w, 3), dtype=torch.float64, device="cuda:0")
        prm = P.params(w, h, 4)
        ctx.render_device(prm, acc.data_ptr(), dev.data_ptr(), 0)
        ctx.sync_stats()
        ctx.render_device(prm, acc.data_ptr(), host.data_ptr(), 0)
        ctx.sync_stats()
        torch.cuda.synchronize()
        assert np.array_equal(dev.cpu().numpy(), host.numpy()), (w, h)
        want, rgb, _ = P.render(sph, cam, w, h, 4)
        assert np.array_equal(host.numpy(), rgb), (w, h)
        del host
        ctx.close()


@pytest.mark.parametrize("buf_mb", [None, "1"])
def test_multi_frame_launch_equals_single_frames(knobs, buf_mb):
    """rt_render_device_frames: frame f of a batch is bit for bit the frame of
    seed + f rendered alone (per-frame seeds, frame-major units, one stats
    fold), for a shard of the final scene, in one sample chunk and (1 MB
    buffer) in several chunks whose running sums continue per frame."""
    import torch
    sph = P.scene_random_spheres(1)
    w, h, spp, nf = 64, 40, 12, 5
    cam = P.camera_look_at(aspect=w / h)
    rows = P.rows_owned(h, 1, 3)
    if buf_mb:
        knobs("sample_buf_mb", int(buf_mb))
    ctx = P.Context(0)
    ctx.set_scene(sph, cam)
    acc = torch.zeros((nf, rows, w, 3), dtype=torch.float64, device="cuda:0")
    rgb = torch.zeros((nf, rows, w, 3), dtype=torch.uint8, device="cuda:0")
    prm = P.params(w, h, spp, 50, 7, 1, 3)
    ctx.render_device_frames(prm, nf, [acc[f].data_ptr() for f in range(nf)],
                             [rgb[f].data_ptr() for f in range(nf)])
    st = ctx.sync_stats()
    torch.cuda.synchronize()
    rays = 0
    for f in range(nf):
        want, wrgb, ws = P.render(sph, cam, w, h, spp, 50, 7 + f, row_offset=1, row_stride=3)
        assert np.array_equal(bits(acc[f].cpu().numpy()), bits(want)), f
        assert np.array_equal(rgb[f].cpu().numpy(), wrgb), f
        rays += ws["rays"]
    assert st["rays"] == rays and st["samples"] == nf * rows * w * spp
    # a NULL entry (frame 2 without bytes) and no accumulator array
    ctx.render_device_frames(prm, 3, None, [rgb[0].data_ptr(), 0, rgb[1].data_ptr()])
    ctx.sync_stats()
    torch.cuda.synchronize()
    _, r0, _ = P.render(sph, cam, w, h, spp, 50, 7, row_offset=1, row_stride=3)
    _, r2, _ = P.render(sph, cam, w, h, spp, 50, 9, row_offset=1, row_stride=3)
    assert np.array_equal(rgb[0].cpu().numpy(), r0) and np.array_equal(rgb[1].cpu().numpy(), r2)
    with pytest.raises(RuntimeError):
        ctx.render_device_frames(prm, 33)
    ctx.close()


@pytest.mark.parametrize("fail_at", ["0", "1"])
def test_render_after_a_failure_mid_render(oracle_mod, knobs, fail_at):
    """A render that fails after a trace launch and before its reduce (the
    rt_debug_fail_after_trace hook stands in for a HIP error there) leaves the
    queue heads and counter sets non-zero: the context is marked dirty, and
    the next render re-zeroes them first and is bit-exact with exact counts.
    fail_at 1: the second of three sample chunks (1 MB sample buffer)."""
    import torch
    sph = oracle_mod.scene_random_spheres(1)
    w, h, spp = 48, 32, 150
    cam = oracle_mod.camera_look_at(aspect=w / h)
    knobs("sample_buf_mb", 1)  # 68 samples of 1536 pixels: chunks of 52, 52, 46
    ctx = P.Context(0)
    ctx.set_scene(sph, cam)
    acc = torch.zeros((h, w, 3), dtype=torch.float64, device="cuda:0")
    ctx.debug_fail_after_trace(int(fail_at))
    with pytest.raises(RuntimeError):
        ctx.render_device(P.params(w, h, spp, 50, 3), acc.data_ptr())
    failed = ctx.sync_stats()  # waits for the part that was enqueued
    # a failed render reports nothing (no stale timings or counts)
    assert failed["kernel_ms"] == 0.0 and failed["total_ms"] == 0.0 and failed["rays"] == 0
    # the hook is one-shot: this render runs in full
    ctx.render_device(P.params(w, h, spp, 50, 3), acc.data_ptr())
    st = ctx.sync_stats()
    want, _, rays = oracle_mod.render(sph, cam, w, h, spp, 50, 3, threads=8)
    assert np.array_equal(bits(acc.cpu().numpy()), bits(want))
    assert st["rays"] == rays and st["samples"] == w * h * spp
    ctx.close()


def test_multi_frame_overlapping_buffers_keep_frame_order():
    """Frames whose accumulator / byte blocks overlap (a stride below one
    frame) are not reduced concurrently: the per-frame reduces
    run in frame order, so each later frame overwrites the overlap as a
    sequence of one-frame renders would."""
    import torch
    sph = P.scene_random_spheres(1)
    w, h, spp, nf = 32, 16, 4, 3
    cam = P.camera_look_at(aspect=w / h)
    P3 = w * h * 3
    half = P3 // 2  # frame f starts half a frame after frame f - 1
    acc = torch.zeros(half * (nf - 1) + P3, dtype=torch.float64, device="cuda:0")
    rgb = torch.zeros(half * (nf - 1) + P3, dtype=torch.uint8, device="cuda:0")
    ctx = P.Context(0)
    ctx.set_scene(sph, cam)
    ctx.render_device_frames(P.params(w, h, spp, 50, 11), nf,
                             [acc.data_ptr() + 8 * half * f for f in range(nf)],
                             [rgb.data_ptr() + half * f for f in range(nf)])
    ctx.sync_stats()
    torch.cuda.synchronize()
    want_acc = np.zeros(acc.shape, dtype=np.float64)
    want_rgb = np.zeros(rgb.shape, dtype=np.uint8)
    for f in range(nf):
        a, r, _ = P.render(sph, cam, w, h, spp, 50, 11 + f)
        want_acc[half * f:half * f + P3] = a.reshape(-1)
        want_rgb[half * f:half * f + P3] = r.reshape(-1)
    assert np.array_equal(bits(acc.cpu().numpy()), bits(want_acc))
    assert np.array_equal(rgb.cpu().numpy(), want_rgb)
    ctx.close()
