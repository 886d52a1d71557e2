"""Host-buffer outputs of the one-shot entries (include/rt.h rt_host_alloc,
DESIGN.md §7 "Host buffers"): page-locked frames are written by the device
directly (psrt_reduce across the link), pageable ones by copy; both hold the
same bits, for one chunk and several, for shards and device groups."""
import numpy as np
import pytest

from conftest import bits

import petershirleyraytracer_amd as P

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cam():
    return P.camera_look_at(aspect=96 / 64)


def test_pinned_outputs_equal_pageable(final_scene, cam):
    want, wrgb, ws = P.render(final_scene, cam, 96, 64, 8, seed=3)
    acc = P.host_array((64, 96, 3))
    rgb = P.host_array((64, 96, 3), np.uint8)
    acc[:] = 7.0  # stale contents: every element must be written
    rgb[:] = 9
    a2, r2, st = P.render(final_scene, cam, 96, 64, 8, seed=3, out=(acc, rgb))
    assert a2 is acc and r2 is rgb
    assert np.array_equal(bits(acc), bits(want)) and np.array_equal(rgb, wrgb)
    assert st["rays"] == ws["rays"]
    # reused for another seed, then the first again
    P.render(final_scene, cam, 96, 64, 8, seed=4, out=(acc, rgb))
    assert not np.array_equal(bits(acc), bits(want))
    P.render(final_scene, cam, 96, 64, 8, seed=3, out=(acc, None))
    assert np.array_equal(bits(acc), bits(want))


def test_pinned_outputs_several_chunks_and_shard(final_scene, cam, knobs):
    """The running sums of a multi-chunk frame live in the caller's pinned
    buffer (read back across the link by each chunk's reduce)."""
    want, wrgb, _ = P.render(final_scene, cam, 96, 64, 64, seed=1, row_offset=1, row_stride=3)
    knobs("sample_buf_mb", 1)  # 22 rows x 96 px x 64 samples x 10 B: 3 chunks
    acc = P.host_array(want.shape)
    rgb = P.host_array(want.shape, np.uint8)
    P.render(final_scene, cam, 96, 64, 64, seed=1, row_offset=1, row_stride=3, out=(acc, rgb))
    assert np.array_equal(bits(acc), bits(want)) and np.array_equal(rgb, wrgb)


def test_pinned_only_bytes_and_pageable_sums(final_scene, cam):
    """Mixed outputs: pageable sums (copied) beside pinned bytes (written
    directly), and pinned bytes with no sums at all."""
    want, wrgb, _ = P.render(final_scene, cam, 96, 64, 8, seed=2)
    rgb = P.host_array((64, 96, 3), np.uint8)
    acc = np.zeros((64, 96, 3))
    P.render(final_scene, cam, 96, 64, 8, seed=2, out=(acc, rgb))
    assert np.array_equal(bits(acc), bits(want)) and np.array_equal(rgb, wrgb)


def test_group_into_pinned(final_scene, cam):
    want, wrgb, _ = P.render(final_scene, cam, 96, 64, 8, seed=5)
    g = P.DeviceGroup([0, 0, 0])
    g.set_scene(final_scene, cam)
    acc = P.host_array((64, 96, 3))
    rgb = P.host_array((64, 96, 3), np.uint8)
    g.render(96, 64, 8, seed=5, out=(acc, rgb))
    g.close()
    assert np.array_equal(bits(acc), bits(want)) and np.array_equal(rgb, wrgb)


def test_row_pitch_shards_assemble_one_frame(final_scene, cam):
    """rt_context_set_row_pitch: three contexts render the shards r::3 with
    their rows 3 x W x 3 apart, straight into one frame (device memory for the
    sums, page-locked host memory for the bytes): the frame equals a
    one-context render bit for bit."""
    import torch
    want, wrgb, _ = P.render(final_scene, cam, 96, 64, 8, seed=7)
    W3 = 96 * 3
    acc = torch.zeros((64, 96, 3), dtype=torch.float64, device="cuda")
    rgb = P.host_array((64, 96, 3), np.uint8)
    ctxs = [P.Context(0) for _ in range(3)]
    for r, c in enumerate(ctxs):
        c.set_scene(final_scene, cam)
        c.set_row_pitch(3 * W3, 3 * W3)
        c.render_device(P.params(96, 64, 8, 50, 7, r, 3), acc.data_ptr() + r * W3 * 8,
                        rgb.ctypes.data + r * W3)
    for c in ctxs:
        c.sync_stats()
    torch.cuda.synchronize()
    assert np.array_equal(bits(acc.cpu().numpy()), bits(want)) and np.array_equal(rgb, wrgb)
    # rows closer than one row apart are an error, so are pitches with materials
    from petershirleyraytracer_amd import _lib
    with pytest.raises(_lib.RtError, match="row pitch"):
        ctxs[0].set_row_pitch(10, 0)
        ctxs[0].render_device(P.params(96, 64, 8, 50, 7, 0, 3), acc.data_ptr(), 0)
    for c in ctxs:
        c.close()


def test_render_bytes_only(final_scene, cam):
    """out=(None, rgb8): rt_render with no accum buffer (the reference main()'s
    output): the sums stay on the device and the bytes equal a full render's,
    into page-locked and pageable arrays alike."""
    want, wrgb, ws = P.render(final_scene, cam, 96, 64, 8, seed=4)
    for rgb in (P.host_array((64, 96, 3), np.uint8), np.zeros((64, 96, 3), np.uint8)):
        acc, got, st = P.render(final_scene, cam, 96, 64, 8, seed=4, out=(None, rgb))
        assert acc is None and got is rgb and np.array_equal(rgb, wrgb)
        assert st["rays"] == ws["rays"]
    with pytest.raises(ValueError):
        P.render(final_scene, cam, 96, 64, 8, seed=4, out=(None, None))
