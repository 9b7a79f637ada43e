"""Multi-GPU inside the boundary (include/prt.h prt_shard_* / prt_create_group) on one GPU.

A local group puts several shards on one device (prt_create_group with a repeated device ordinal): each member
renders its round-robin pixel tiles on its own stream and member 0 gathers and untiles, so the decomposition
of the N-GPU frame is checked here bit for bit against the single-context frame.  The RCCL transport is
exercised with a world-1 communicator (RCCL refuses two ranks on one device), and the caller-side transport
(prt.tiles.ShardedFrame) over a world-1 torch "nccl" group without stats (no host synchronisation between the
tile render, the gather and the untile)."""
import socket

import numpy as np
import pytest

from helpers import gpu_scene
from prt import scenes

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,post", [(2, False), (3, True), (5, False)])
def test_group_matches_single(gpu_ctx, world, post):
    import prt
    sd = scenes.multi_instance(scenes.config_small(60, 40))
    W, H, ts = 100, 70, 16
    pf = prt.postfx_preset(0, color_grading=(1.0, 0.9, 1.2, 1.0)) if post else None
    gpu_scene(gpu_ctx, sd, W, H)
    gpu_ctx.set_postfx(pf)
    try:
        a_full, r_full, s_full = gpu_ctx.render(W, H, 4, 3)
        a2_full, r2_full, _ = gpu_ctx.render(W, H, 4, 3, frame_index=2)  # accumulating second call
    finally:
        gpu_ctx.set_postfx(None)
    g = prt.Context(group=[0] * world, tile=ts)
    try:
        si = g.shard_info()
        assert (si.rank, si.world, si.tile_size, si.transport) == (0, world, ts, prt._lib.SHARD_GROUP)
        gpu_scene(g, sd, W, H)
        g.set_postfx(pf)
        a, r, st = g.render(W, H, 4, 3)
        assert np.array_equal(a, a_full) and np.array_equal(r, r_full)
        assert s_full.paths == W * H * 4  # camera paths of in-image pixels only (not the tiles' overhang)
        assert (st.segments, st.shadow_rays, st.paths) == (s_full.segments, s_full.shadow_rays, s_full.paths)
        assert st.ranks == world
        a2, r2, _ = g.render(W, H, 4, 3, frame_index=2)
        assert np.array_equal(a2, a2_full) and np.array_equal(r2, r2_full)
    finally:
        g.close()


def test_group_full_size_c4_world8(gpu_ctx):
    """The driver's N = 8 decomposition of the bench frame (C4, 1920x1080, 4 spp, depth 4, 32x32 tiles) as one
    8-member group on this GPU, device outputs, no stats (the frames of the 8 members run concurrently on 8
    streams): bit-identical to the single-GPU frame."""
    import torch
    import prt
    sd = scenes.config_c4()
    W, H = 1920, 1080
    gpu_scene(gpu_ctx, sd, W, H)
    a_full, r_full, s_full = gpu_ctx.render(W, H, 4, 4)
    g = prt.Context(group=[0] * 8, tile=32)
    try:
        gpu_scene(g, sd, W, H)
        avg = torch.zeros((H * W, 4), dtype=torch.float32, device="cuda")
        rgb = torch.zeros(H * W, dtype=torch.int32, device="cuda")
        g.render(W, H, 4, 4, avg=avg.data_ptr(), rgb8=rgb.data_ptr(), device_out=True, stats=False)
        torch.cuda.synchronize()
        assert np.array_equal(avg.cpu().numpy(), a_full)
        assert np.array_equal(rgb.cpu().numpy().view(np.uint32), r_full)
        g.reset_accumulation(full=True)
        _, _, st = g.render(W, H, 4, 4)
        assert (st.segments, st.shadow_rays) == (s_full.segments, s_full.shadow_rays) and st.ranks == 8
    finally:
        g.close()


def test_group_refuses_aberration(gpu_ctx):
    import prt
    sd = scenes.config_small(20, 20)
    g = prt.Context(group=[0, 0], tile=16)
    try:
        gpu_scene(g, sd, 48, 32)
        g.set_postfx(prt.postfx_preset(1))  # P1: aberration -1
        with pytest.raises(prt.PrtError):
            g.render(48, 32, 2, 2)
    finally:
        g.close()


def test_rccl_world1_matches_single(gpu_ctx):
    """prt_shard_unique_id + prt_shard_init_rccl (the context owns the communicator): a world-1 RCCL shard renders
    through the ncclGather path and equals the unsharded frame."""
    import prt
    sd = scenes.multi_instance(scenes.config_small(50, 40))
    W, H = 90, 60
    gpu_scene(gpu_ctx, sd, W, H)
    a_full, r_full, s_full = gpu_ctx.render(W, H, 4, 3)
    c = prt.Context(0)
    try:
        c.shard_rccl(prt.Context.shard_unique_id(), 0, 1, 32)
        si = c.shard_info()
        assert (si.rank, si.world, si.transport) == (0, 1, prt._lib.SHARD_RCCL)
        gpu_scene(c, sd, W, H)
        a, r, st = c.render(W, H, 4, 3)
        assert np.array_equal(a, a_full) and np.array_equal(r, r_full)
        assert (st.segments, st.shadow_rays) == (s_full.segments, s_full.shadow_rays)
        with pytest.raises(prt.PrtError):
            c.shard_rccl(prt.Context.shard_unique_id(), 0, 1, 32)  # already sharded
    finally:
        c.close()


def test_sharded_frame_torch_world1_no_stats(gpu_ctx):
    """prt.tiles.ShardedFrame over a world-1 torch "nccl" group with stats off: the context follows torch's
    stream, so tile render -> dist.gather -> untile are stream-ordered without a host sync."""
    import torch
    import torch.distributed as dist
    import prt
    sd = scenes.multi_instance(scenes.config_small(50, 40))
    W, H, ts = 96, 64, 32
    gpu_scene(gpu_ctx, sd, W, H)
    a_full, r_full, _ = gpu_ctx.render(W, H, 4, 3)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    c = prt.Context(0)
    try:
        gpu_scene(c, sd, W, H)
        shard = prt.tiles.ShardedFrame(c, dist, W, H, ts, device="cuda")
        avg = torch.zeros((H * W, 4), dtype=torch.float32, device="cuda")
        rgb = torch.zeros(H * W, dtype=torch.int32, device="cuda")
        for _ in range(2):  # the second frame reuses the tile / gather buffers while nothing waits on the host
            c.reset_accumulation(full=True)
            shard.render(4, 3, avg.data_ptr(), rgb.data_ptr(), stats=False)
        torch.cuda.synchronize()
        assert np.array_equal(avg.cpu().numpy(), a_full)
        assert np.array_equal(rgb.cpu().numpy().view(np.uint32), r_full)
    finally:
        c.close()
        dist.destroy_process_group()
