"""Multi-rank frame sharding on CPU (gloo): the tile partition, the one gather per frame and the untile of
prt.tiles.ShardedFrame, with the per-rank render stood in by the oracle (each rank contributes exactly the
pixels its tile map owns).  The GPU path of the same code (prt_render_tiles / prt_untile kernels) is
covered by tests/test_gpu_parity.py::test_tiles_match_full_frame; bench.py --gpus N drives it over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

W, H, TILE, SPP, BOUNCES = 72, 40, 16, 2, 3


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _OracleRankCtx:
    """Stands in for prt.Context on a GPU-less rank: render_tiles fills the rank's tile buffer from an oracle
    frame through prt_tile_pixel_map; untile scatters with the host mirror of prt_untile."""

    def __init__(self, frame):
        self.frame = frame
        self.shard = None

    def render_tiles(self, width, height, spp, bounces, tile, rank, world, ptr, **kw):
        from prt import tiles
        assert ptr == self.shard.tiles.data_ptr()
        m = tiles.tile_pixel_map(width, height, tile, rank, world)
        buf = np.zeros((m.size, 4), np.float32)
        buf[m >= 0] = self.frame[m[m >= 0]]
        self.shard.tiles.copy_(torch.from_numpy(buf))
        return None

    def finish(self):  # prt_finish: nothing in flight on a CPU rank
        pass

    def untile(self, gathered_ptr, width, height, tile, world, avg_ptr, rgb8_ptr):
        from prt import tiles
        assert gathered_ptr == self.shard.gathered.data_ptr()
        self.out = tiles.untile_host(self.shard.gathered.numpy(), width, height, tile)


def _worker(rank, world, port, frame, result_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from prt import tiles
        ctx = _OracleRankCtx(frame)
        shard = tiles.ShardedFrame(ctx, dist, W, H, TILE, device="cpu")
        ctx.shard = shard
        shard.render(SPP, BOUNCES, 0, 0)
        if rank == 0:
            result_q.put(ctx.out)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_frame_gloo(oracle_mod, world):
    from prt import scenes
    sd = scenes.config_small(30, 20)
    osc = oracle_mod.OracleScene(sd, W, H)
    frame, _, _, _ = osc.render(W, H, spp=SPP, bounces=BOUNCES)
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    port = _free_port()
    procs = [ctxm.Process(target=_worker, args=(r, world, port, frame, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert np.array_equal(out, frame)


def test_tile_maps_partition_the_image():
    from prt import tiles
    for world in (1, 2, 3, 8):
        seen = np.zeros(1920 * 1080, np.int32)
        for r in range(world):
            m = tiles.tile_pixel_map(1920, 1080, 32, r, world)
            assert m.size == tiles.tile_buffer_pixels(1920, 1080, 32, world)
            np.add.at(seen, m[m >= 0], 1)
        assert np.all(seen == 1)
