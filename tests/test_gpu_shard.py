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


@pytest.mark.parametrize("caller_stream", ["default", "side"])
def test_sharded_frame_torch_world1_no_stats(gpu_ctx, caller_stream):
    """prt.tiles.ShardedFrame over a world-1 torch "nccl" group with stats off: tile render -> dist.gather ->
    untile run on the frame's own stream without a host sync, ordered after the caller's stream and before its
    later reads, whether the caller is on the legacy default stream or a side stream."""
    import contextlib

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
    side = torch.cuda.Stream() if caller_stream == "side" else None
    try:
        gpu_scene(c, sd, W, H)
        with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
            shard = prt.tiles.ShardedFrame(c, dist, W, H, ts, device="cuda")
            avg = torch.zeros((H * W, 4), dtype=torch.float32, device="cuda")
            rgb = torch.zeros(H * W, dtype=torch.int32, device="cuda")
            for _ in range(2):  # the second frame reuses the tile / gather buffers while nothing waits on the host
                c.reset_accumulation(full=True)
                shard.render(4, 3, avg.data_ptr(), rgb.data_ptr(), stats=False)
            out_avg, out_rgb = avg.clone(), rgb.clone()  # on the caller's stream: ordered after the untile
        torch.cuda.synchronize()
        assert np.array_equal(out_avg.cpu().numpy(), a_full)
        assert np.array_equal(out_rgb.cpu().numpy().view(np.uint32), r_full)
    finally:
        c.close()
        dist.destroy_process_group()


def _visible_devices():
    import torch
    return torch.cuda.device_count()


@pytest.mark.skipif("_visible_devices() < 2", reason="needs two visible GPUs (cross-device group / RCCL world 2)")
def test_group_two_devices_matches_single(gpu_ctx):
    """A local group over two devices (prt_create_group([0, 1])): member 1 renders on device 1 and its tile
    buffer reaches member 0 by hipMemcpyPeerAsync, ordered by the cross-device events."""
    import prt
    sd = scenes.multi_instance(scenes.config_small(60, 40))
    W, H, ts = 100, 70, 16
    gpu_scene(gpu_ctx, sd, W, H)
    a_full, r_full, s_full = gpu_ctx.render(W, H, 4, 3)
    g = prt.Context(group=[0, 1], tile=ts)
    try:
        gpu_scene(g, sd, W, H)
        for _ in range(2):  # the second frame's peer copy waits for the first frame's untile
            g.reset_accumulation(full=True)
            a, r, st = g.render(W, H, 4, 3)
            assert np.array_equal(a, a_full) and np.array_equal(r, r_full)
            assert (st.segments, st.shadow_rays) == (s_full.segments, s_full.shadow_rays)
    finally:
        g.close()


def _rccl_rank(rank, world, port, out_path):
    import torch
    import torch.distributed as dist
    import prt
    torch.cuda.set_device(rank)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                            device_id=torch.device("cuda", rank))
    sd = scenes.multi_instance(scenes.config_small(60, 40))
    W, H = 100, 70
    c = prt.Context(rank)
    try:
        gpu_scene(c, sd, W, H)
        si = prt.tiles.join_rccl(c, dist, 16)
        assert (si.rank, si.world) == (rank, world)
        avg = torch.zeros((H * W, 4), dtype=torch.float32, device="cuda")
        rgb = torch.zeros(H * W, dtype=torch.int32, device="cuda")
        _, _, st = c.render(W, H, 4, 3, avg=avg.data_ptr(), rgb8=rgb.data_ptr(), device_out=True)
        r = torch.tensor([st.segments, st.shadow_rays], dtype=torch.float64, device="cuda")
        dist.all_reduce(r)
        if rank == 0:
            np.savez(out_path, avg=avg.cpu().numpy(), rgb=rgb.cpu().numpy().view(np.uint32),
                     rays=r.cpu().numpy())
    finally:
        c.close()
        dist.destroy_process_group()


@pytest.mark.skipif("_visible_devices() < 2", reason="needs two visible GPUs (RCCL refuses two ranks on one device)")
def test_rccl_world2_matches_single(gpu_ctx, tmp_path):
    """Two processes, one GPU each, one RCCL communicator inside the contexts: rank 1's tiles reach rank 0 through
    ncclGather (NULL receive buffer on the non-root rank) and rank 0's frame equals the single-context frame."""
    import torch.multiprocessing as mp
    sd = scenes.multi_instance(scenes.config_small(60, 40))
    W, H = 100, 70
    gpu_scene(gpu_ctx, sd, W, H)
    a_full, r_full, s_full = gpu_ctx.render(W, H, 4, 3)
    out = str(tmp_path / "rank0.npz")
    mp.spawn(_rccl_rank, args=(2, _free_port(), out), nprocs=2, join=True)
    z = np.load(out)
    assert np.array_equal(z["avg"], a_full) and np.array_equal(z["rgb"], r_full)
    assert tuple(int(x) for x in z["rays"]) == (s_full.segments, s_full.shadow_rays)


def test_failed_group_frame_returns_error_and_next_frame_exact(gpu_ctx, monkeypatch):
    """A member's render fails (PRT_FAIL_RENDER=<member>, raised in prepare_render before any render work is
    enqueued): the group call returns the error, no member's accumulation advanced, and the next frames equal the
    single-context frames of the same sequence without the failed call."""
    import prt
    sd = scenes.multi_instance(scenes.config_small(60, 40))
    W, H, ts = 100, 70, 16
    gpu_scene(gpu_ctx, sd, W, H)
    a1, r1, _ = gpu_ctx.render(W, H, 4, 3)
    a2, r2, _ = gpu_ctx.render(W, H, 4, 3, frame_index=2)  # accumulating
    g = prt.Context(group=[0] * 3, tile=ts)
    try:
        gpu_scene(g, sd, W, H)
        a, r, _ = g.render(W, H, 4, 3)
        assert np.array_equal(a, a1) and np.array_equal(r, r1)
        monkeypatch.setenv("PRT_FAIL_RENDER", "2")
        with pytest.raises(prt.PrtError, match="injected"):
            g.render(W, H, 4, 3, frame_index=2)
        monkeypatch.delenv("PRT_FAIL_RENDER")
        a, r, _ = g.render(W, H, 4, 3, frame_index=2)
        assert np.array_equal(a, a2) and np.array_equal(r, r2)
    finally:
        g.close()


def test_failed_rccl_frame_posts_gather_and_next_frame_exact(gpu_ctx, monkeypatch):
    """RCCL world 1: the failing rank still posts its (zero) part of the frame's ncclGather (post_zero_gather,
    so peers never block), returns the error, and the next frame is exact."""
    import prt
    sd = scenes.multi_instance(scenes.config_small(50, 40))
    W, H = 90, 60
    gpu_scene(gpu_ctx, sd, W, H)
    a1, r1, _ = gpu_ctx.render(W, H, 4, 3)
    a2, r2, _ = gpu_ctx.render(W, H, 4, 3, frame_index=2)
    c = prt.Context(0)
    try:
        c.shard_rccl(prt.Context.shard_unique_id(), 0, 1, 32)
        gpu_scene(c, sd, W, H)
        a, r, _ = c.render(W, H, 4, 3)
        assert np.array_equal(a, a1) and np.array_equal(r, r1)
        monkeypatch.setenv("PRT_FAIL_RENDER", "0")
        with pytest.raises(prt.PrtError, match="injected"):
            c.render(W, H, 4, 3, frame_index=2)
        monkeypatch.delenv("PRT_FAIL_RENDER")
        a, r, st = c.render(W, H, 4, 3, frame_index=2)  # the zero gather completed: the stream is not stuck
        assert np.array_equal(a, a2) and np.array_equal(r, r2)
        assert st.stack_overflows == 0
    finally:
        c.close()


def test_frame_above_pass_limit_refused(gpu_ctx):
    """A frame (of one shard) above 2^27 pixels would overflow the 29-bit item field of the shadow-queue entries
    (prt_wave2.hip kShIndexMask): refused with PRT_ERR_UNSUPPORTED before any allocation."""
    import prt
    sd = scenes.config_small(20, 20)
    gpu_scene(gpu_ctx, sd, 64, 48)
    with pytest.raises(prt.PrtError, match="2\\^27"):
        gpu_ctx.render(16384, 16384, 2, 1, device_out=True, stats=False)  # no output buffers
    a, _, _ = gpu_ctx.render(64, 48, 2, 2)  # the context is still usable
    assert np.isfinite(a).all()
