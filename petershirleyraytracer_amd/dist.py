"""Multi-GPU sharding of the frame: one process per GPU, interleaved rows.

Rank g of G owns output rows r = g, g+G, g+2G, ... (rt_params.row_offset = g,
row_stride = G). Every (pixel, sample) is independent under the counter RNG,
so the shards need no exchange while rendering; the one exchange step is the
framebuffer's assembly on rank 0: on one node, in a page-locked frame in
shared host memory that every rank writes its rows into (HostFrames), or by
a gather to rank 0 (RCCL over xGMI with backend "nccl", gloo on CPU).
Interleaving balances the load: contiguous row bands of the final scene
cost 0.15-1.32x the mean. The gathered frame is bit-identical
for any G because each pixel's accumulation never leaves its lane.
"""
from __future__ import annotations

import ctypes as C
import uuid
from multiprocessing import shared_memory
from typing import Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist


def shard(rank: int, world: int) -> Tuple[int, int]:
    """(row_offset, row_stride) of a rank."""
    if not (0 <= rank < world):
        raise ValueError(f"rank {rank} outside world {world}")
    return rank, world


def rows_owned(height: int, rank: int, world: int) -> int:
    if rank >= height:
        return 0
    return (height - 1 - rank) // world + 1


def gather_frame(local: torch.Tensor, height: int, rank: int, world: int,
                 dst: int = 0) -> Optional[torch.Tensor]:
    """One frame: `gather_frames` of a [rows_owned, W, C] block."""
    if world == 1:
        return local
    out = gather_frames(local.unsqueeze(0), height, rank, world, dst)
    return None if out is None else out[0]


def gather_frames(local: torch.Tensor, height: int, rank: int, world: int,
                  dst: int = 0) -> Optional[torch.Tensor]:
    """Gather per-rank row blocks [B, rows_owned, W, C] of B frames into the
    full frames [B, height, W, C] on rank `dst` (None elsewhere).

    One gather to `dst` of blocks padded to ceil(height/world) rows, for all B
    frames at once (one collective and one de-interleave per rank instead of
    one per frame): only the destination receives them (an all_gather would
    send every block to every rank). A rank that owns no rows (world > height)
    sends an all-padding block. The destination then de-interleaves."""
    if world == 1:
        return local
    return _gather_blocks(local, height, rank, world, dst)


def _gather_blocks(local: torch.Tensor, height: int, rank: int, world: int,
                   dst: int) -> Optional[torch.Tensor]:
    """The collective of `gather_frames` (also run at world 1 by the GPU test
    that drives RCCL's gather on device frames on a one-GPU box)."""
    max_rows = rows_owned(height, 0, world)
    mine = rows_owned(height, rank, world)
    if local.dim() != 4 or local.shape[1] != mine:
        raise ValueError(f"rank {rank} holds {tuple(local.shape)}, owns {mine} rows")
    nb, w, ch = local.shape[0], local.shape[2], local.shape[3]
    padded = local.new_zeros((nb, max_rows, w, ch))
    if mine:
        padded[:, :mine] = local
    # gloo's gather takes host tensors only (the N > 1 rehearsal on one GPU
    # runs gloo over device frames): stage through host memory there
    host = dist.get_backend() == "gloo" and padded.device.type != "cpu"
    send = padded.cpu() if host else padded
    parts = [torch.empty_like(send) for _ in range(world)] if rank == dst else None
    dist.gather(send, parts, dst=dst)
    if host and rank == dst:
        parts = [p.to(local.device) for p in parts]
    if rank != dst:
        return None
    frames = local.new_empty((nb, height, w, ch))
    for r in range(world):
        n = rows_owned(height, r, world)
        if n:
            frames[:, r::world] = parts[r][:, :n]
    return frames


class HostFrames:
    """Frames assembled in place in page-locked host memory shared by the
    ranks of one node (DESIGN.md §5 "Frame to host"): rank 0 creates a POSIX
    shared-memory segment of `nframes` frames [H, W, 3] uint8, every rank maps
    it and page-locks it (rt_host_register), and each rank's psrt_reduce writes
    its interleaved rows straight into it (rt_context_set_row_pitch: rows
    G * W * 3 bytes apart). Every rank's bytes cross its own GPU's link, in
    parallel; no collective and no device-to-host copy on rank 0. The frames
    are complete on every rank once all ranks' renders are done (a barrier).
    Collective: every rank constructs it; close() on every rank."""

    def __init__(self, nframes: int, height: int, width: int, rank: int, world: int):
        from . import _lib
        self._L = _lib.load()
        self.shape = (nframes, height, width, 3)
        self.frame_bytes = height * width * 3
        size = max(1, nframes * self.frame_bytes)
        self.owner = rank == 0
        self.shm = None
        name = [None]
        if self.owner:  # created before its name goes out
            self.shm = shared_memory.SharedMemory(name=f"psrt_{uuid.uuid4().hex[:16]}",
                                                  create=True, size=size)
            name[0] = self.shm.name
        try:
            dist.broadcast_object_list(name, src=0)
            if not self.owner:
                self.shm = shared_memory.SharedMemory(name=name[0], create=False, size=size)
                # the owner unlinks it below: the other ranks' resource trackers
                # must not try again at exit (Python < 3.13 registers attaches too)
                from multiprocessing import resource_tracker
                try:
                    resource_tracker.unregister(self.shm._name, "shared_memory")
                except Exception:
                    pass
            dist.barrier()  # every rank has mapped it before the owner may unlink
        finally:
            if self.owner:
                self.shm.unlink()  # the mappings stay; nothing is left in /dev/shm
        self.frames = np.ndarray(self.shape, dtype=np.uint8, buffer=self.shm.buf)
        self.addr = C.addressof(C.c_ubyte.from_buffer(self.shm.buf))
        # page-locking is per rank (and per device): a failure is reported in
        # `registered` / `error` rather than raised, so the ranks can agree on
        # a fallback together (bench.py) instead of one rank leaving the others
        rc = self._L.rt_host_register(C.c_void_p(self.addr), size)
        self.registered = rc == 0
        self.error = None if self.registered else self._L.rt_last_error().decode(errors="replace")
        self.row_offset, self.row_stride = rank, world

    def rows_ptr(self, f: int, width: int) -> int:
        """Frame f's first row of this rank's shard."""
        return self.addr + f * self.frame_bytes + self.row_offset * width * 3

    def close(self) -> None:
        if getattr(self, "registered", False):
            self._L.rt_host_unregister(C.c_void_p(self.addr))
            self.registered = False
        if getattr(self, "shm", None) is not None:
            self.frames = None
            try:
                self.shm.close()
            except BufferError:
                pass
            self.shm = None
