"""Pixel-tile sharding of one frame over the GPUs of a node (no counterpart in the reference,
whose OpenMP loop over rows, Core/Renderer.cpp:43, is the single-process analogue).

One process per GPU.  Tiles of tile x tile pixels, numbered row-major, go round-robin to the ranks
(rank r: tiles r, r+world, ...).  Every rank renders all samples of its tiles into a compact float4
buffer [local tile][tile*tile] (prt_render_tiles), the buffers meet on rank 0 in ONE RCCL gather per
frame, and rank 0 scatters them back into the W x H image (prt_untile).  Pixels are independent, so
there is no other exchange.  join_rccl puts all of that inside the context (the RCCL communicator is the
context's; prt_render does the tile render, the gather and the untile); ShardedFrame is the same frame
with the gather done by the caller's torch.distributed group.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import check


def tile_buffer_pixels(width: int, height: int, tile: int, world: int) -> int:
    """Elements of each rank's tile buffer (equal on all ranks: rank 0's, the largest)."""
    n = C.c_int64(0)
    check(_lib.load().prt_tile_buffer_pixels(width, height, tile, world, C.byref(n)))
    return n.value


def tile_pixel_map(width: int, height: int, tile: int, rank: int, world: int) -> np.ndarray:
    """Image pixel index (y*W + x) of each element of rank's tile buffer; -1 outside the image."""
    out = np.zeros(tile_buffer_pixels(width, height, tile, world), np.int32)
    check(_lib.load().prt_tile_pixel_map(width, height, tile, rank, world, out.ctypes.data))
    return out


def untile_host(gathered: np.ndarray, width: int, height: int, tile: int) -> np.ndarray:
    """Host mirror of prt_untile's scatter: gathered [world][per][4] -> [W*H][4]."""
    world = gathered.shape[0]
    img = np.zeros((width * height, gathered.shape[-1]), gathered.dtype)
    for r in range(world):
        m = tile_pixel_map(width, height, tile, r, world)
        ok = m >= 0
        img[m[ok]] = gathered[r][ok]
    return img


def join_rccl(ctx, dist, tile: int = 32):
    """Shard `ctx` over the ranks of a torch.distributed group, inside the boundary: rank 0 makes the RCCL
    id (prt_shard_unique_id), the group carries its bytes to the other ranks, and every rank's context joins
    the communicator it then owns (prt_shard_init_rccl).  After this, ctx.render() on every rank renders
    that rank's tiles and leaves the whole frame in rank 0's outputs."""
    rank, world = dist.get_rank(), dist.get_world_size()
    box = [ctx.shard_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(box, src=0)
    ctx.shard_rccl(box[0], rank, world, tile)
    return ctx.shard_info()


class ShardedFrame:
    """The caller-side transport: one frame split over a torch.distributed group (prt_render_tiles, one
    dist.gather to rank 0, prt_untile) -- what a host whose framework owns the collectives uses instead of
    join_rccl.

    ctx: this rank's prt.Context (its own GPU); tiles and gathered buffers live on that GPU.  On a GPU the
    frame runs on a dedicated torch stream that the context is moved onto: the tile render, the gather
    (queued there by torch) and the untile are ordered on it without a host sync.  A dedicated stream, not
    torch's current one, because the current one may be the legacy default stream, which the context's
    non-blocking stream (prt_set_stream(NULL)) does not order against.  The stream waits for the caller's
    current stream on entry and the caller's stream waits for it on exit.
    render() returns this rank's prt_stats; rank 0's avg/rgb8 device buffers hold the full frame."""

    def __init__(self, ctx, dist, width: int, height: int, tile: int = 32, device=None):
        import torch
        self.ctx, self.dist, self.W, self.H, self.tile = ctx, dist, width, height, tile
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.stream = None
        if device is not None and torch.device(device).type == "cuda":
            self.stream = torch.cuda.Stream(device=device)
            ctx.set_stream(self.stream.cuda_stream)
        per = tile_buffer_pixels(width, height, tile, self.world)
        self.tiles = torch.zeros((per, 4), dtype=torch.float32, device=device)
        self.gathered = (torch.zeros((self.world, per, 4), dtype=torch.float32, device=device)
                         if self.rank == 0 else None)

    def render(self, spp, bounces, avg_ptr, rgb8_ptr, frame_index=0, flags=_lib.FLAGS_DEFAULT, stats=True):
        import torch
        if self.stream is None:
            return self._render(spp, bounces, avg_ptr, rgb8_ptr, frame_index, flags, stats)
        caller = torch.cuda.current_stream(self.stream.device)
        self.stream.wait_stream(caller)  # the caller's writes (buffers, scene updates) come first
        with torch.cuda.stream(self.stream):
            st = self._render(spp, bounces, avg_ptr, rgb8_ptr, frame_index, flags, stats)
        caller.wait_stream(self.stream)  # the caller's later reads of avg / rgb8 come after the untile
        return st

    def _render(self, spp, bounces, avg_ptr, rgb8_ptr, frame_index, flags, stats):
        st = self.ctx.render_tiles(self.W, self.H, spp, bounces, self.tile, self.rank, self.world,
                                   self.tiles.data_ptr(), flags=flags, frame_index=frame_index, stats=stats)
        # with frames in flight the tile render may still be on an internal stream: the gather torch queues on
        # the context stream must come after it (prt_finish joins it there, no host wait)
        self.ctx.finish()
        self.dist.gather(self.tiles, list(self.gathered.unbind(0)) if self.rank == 0 else None, dst=0)
        if self.rank == 0:
            self.ctx.untile(self.gathered.data_ptr(), self.W, self.H, self.tile, self.world, avg_ptr, rgb8_ptr)
        return st
