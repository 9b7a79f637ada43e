"""Frames in flight (include/prt.h prt_set_frames_in_flight, ABI 9): with 2 frames in flight a prt_render with
device outputs enqueues its wavefront chain on one of two internal streams, so consecutive calls overlap, while the
accumulation (the reference's progressive mean, Core/Renderer.cpp:81-104) and a sharded frame's gather stay in call
order.  Every frame must equal the one-at-a-time render bit for bit: outputs, ray totals, through instance updates
(the instance BVH rebuilt between frames; an update writes the next copy of the instance state while the frames in
flight read theirs), a camera change with an accumulation reset, a stats call in between, the merged and unmerged
pipelines and the RCCL gather."""
import numpy as np
import pytest

from helpers import gpu_scene
from prt import scenes

pytestmark = pytest.mark.gpu


def _frames(c, sd, W, H, n, moves, stream, materials_at=-1):
    """n accumulating frames with device outputs (one output pair per frame), instance moves before the frames in
    `moves`, mirror materials on every 5th instance before frame `materials_at`, a camera change + accumulation
    reset before frame n - 2 and a stats render at the end."""
    import torch
    import prt
    outs = []
    inst = [(m, np.array(T, np.float32)) for m, T in sd.instances]
    for f in range(n):
        if f in moves:
            inst = [(m, _shift(T, m)) for m, T in inst]
            c.set_instances(inst)
        if f == materials_at:
            c.set_materials([2 if i % 5 == 1 else 0 for i in range(len(inst))])
        if f == n - 2:
            cam = prt.Camera(np.asarray(sd.cam_pos, np.float32) + np.float32(0.25), sd.cam_target,
                             np.float32(W) / np.float32(H))
            c.set_camera(cam)
            c.reset_accumulation(full=False)
        with torch.cuda.stream(stream):
            avg = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
            rgb = torch.zeros(W * H, dtype=torch.int32, device="cuda")
        c.render(W, H, 4, 3, frame_index=2 * f, avg=avg.data_ptr(), rgb8=rgb.data_ptr(), device_out=True,
                 stats=False)
        outs.append((avg, rgb))
    a, r, st = c.render(W, H, 4, 3, frame_index=2 * n)  # host outputs + stats: joins the frames in flight
    torch.cuda.synchronize()
    seg, sh = c.ray_totals(reset=True)
    return [(o.cpu().numpy(), g.cpu().numpy()) for o, g in outs], (a, r, st.segments, st.shadow_rays), (seg, sh)


def _shift(T, m):
    T = T.copy()
    if m == 1:  # the tori move, the heightfield stays
        T[0, 3] += np.float32(0.07)
        T[2, 3] -= np.float32(0.05)
    return T


@pytest.mark.parametrize("merge,flights", [("default", 2), ("default", 4), ("0", 3)])
def test_frames_in_flight_match_one_at_a_time(monkeypatch, merge, flights):
    import torch
    import prt
    if merge == "0":
        monkeypatch.setenv("PRT_MERGE", "0")
    else:
        monkeypatch.delenv("PRT_MERGE", raising=False)
    sd = scenes.instance_field(120, seed=9)  # above 64 instances: the instance BVH is refitted between frames
    W, H, n = 96, 64, 7
    stream = torch.cuda.Stream()
    res = []
    for fl in (1, flights):
        c = prt.Context(0)
        try:
            c.set_stream(stream.cuda_stream)
            gpu_scene(c, sd, W, H)
            c.set_frames_in_flight(fl)
            res.append(_frames(c, sd, W, H, n, {3}, stream))
        finally:
            c.close()
    (f1, last1, tot1), (f2, last2, tot2) = res
    for k, ((a1, r1), (a2, r2)) in enumerate(zip(f1, f2)):
        assert np.array_equal(a1, a2) and np.array_equal(r1, r2), k
    assert np.array_equal(last1[0], last2[0]) and np.array_equal(last1[1], last2[1])
    assert last1[2:] == last2[2:] and tot1 == tot2


@pytest.mark.parametrize("flights,n_inst", [(2, 120), (4, 120), (3, 40)])
def test_frames_in_flight_instance_updates_every_frame(flights, n_inst):
    """Instances moved before every frame and a materials update, with frames in flight: prt_set_instances does not
    join the frames in flight, each update writing the next of flights + 1 copies of the instance state (records,
    refit input, instance BVH) once the frames that read it are done; every frame equals the one-at-a-time render
    (120 instances: the instance BVH, built on the worker thread in stream order; 40: the linear list)."""
    import torch
    import prt
    sd = scenes.instance_field(n_inst, seed=9)
    W, H, n = 96, 64, 9
    stream = torch.cuda.Stream()
    res = []
    for fl in (1, flights):
        c = prt.Context(0)
        try:
            c.set_stream(stream.cuda_stream)
            gpu_scene(c, sd, W, H)
            c.set_frames_in_flight(fl)
            res.append(_frames(c, sd, W, H, n, set(range(1, n)), stream, materials_at=4))
        finally:
            c.close()
    (f1, last1, tot1), (f2, last2, tot2) = res
    for k, ((a1, r1), (a2, r2)) in enumerate(zip(f1, f2)):
        assert np.array_equal(a1, a2) and np.array_equal(r1, r2), k
    assert np.array_equal(last1[0], last2[0]) and np.array_equal(last1[1], last2[1])
    assert last1[2:] == last2[2:] and tot1 == tot2


@pytest.mark.parametrize("flights", [2, 3])
def test_frames_in_flight_outputs_in_stream_order(flights):
    """A call's device outputs are complete in the context stream's order once flights - 1 more calls are enqueued
    (or after prt_finish): a copy enqueued on the caller's stream right then sees the finished frame."""
    import torch
    import prt
    sd = scenes.multi_instance(scenes.config_small(60, 40))
    W, H = 100, 70
    stream = torch.cuda.Stream()
    ref = prt.Context(0)
    c = prt.Context(0)
    try:
        gpu_scene(ref, sd, W, H)
        n = 5
        want = [ref.render(W, H, 4, 3, frame_index=2 * f)[0] for f in range(n)]
        c.set_stream(stream.cuda_stream)
        gpu_scene(c, sd, W, H)
        c.set_frames_in_flight(flights)
        got = {}
        with torch.cuda.stream(stream):
            outs = [torch.zeros((W * H, 4), dtype=torch.float32, device="cuda") for _ in range(n)]
        for f in range(n):
            c.render(W, H, 4, 3, frame_index=2 * f, avg=outs[f].data_ptr(), device_out=True, stats=False)
            k = f - (flights - 1)
            if k >= 0:
                with torch.cuda.stream(stream):
                    got[k] = outs[k].clone()
        c.finish()
        with torch.cuda.stream(stream):
            for k in range(n):
                if k not in got:
                    got[k] = outs[k].clone()
        stream.synchronize()
        for f in range(n):
            assert np.array_equal(got[f].cpu().numpy(), want[f]), f
    finally:
        c.close()
        ref.close()


@pytest.mark.parametrize("flights", [3, 4])
def test_frames_in_flight_rccl_world1(flights):
    """An RCCL shard (world 1: the ncclGather path) with 3 or 4 frames in flight (4: the setting bench.py uses on
    several GPUs, with each chain on cut grids): each call's gather and untile run on its slot's stream after
    the previous call's; through an instance update, a camera change with an accumulation reset and a stats call,
    every frame equals the unsharded one-at-a-time render bit for bit."""
    import torch
    import prt
    sd = scenes.instance_field(120, seed=9)  # above 64 instances: the instance BVH is refitted between frames
    W, H, n = 96, 64, 7
    stream = torch.cuda.Stream()
    res = []
    for fl, shard in ((1, False), (flights, True)):
        c = prt.Context(0)
        try:
            c.set_stream(stream.cuda_stream)
            if shard:
                c.shard_rccl(prt.Context.shard_unique_id(), 0, 1, 32)
            gpu_scene(c, sd, W, H)
            c.set_frames_in_flight(fl)
            res.append(_frames(c, sd, W, H, n, set(range(1, n)), stream))
        finally:
            c.close()
    (f1, last1, tot1), (f2, last2, tot2) = res
    for k, ((a1, r1), (a2, r2)) in enumerate(zip(f1, f2)):
        assert np.array_equal(a1, a2) and np.array_equal(r1, r2), k
    assert np.array_equal(last1[0], last2[0]) and np.array_equal(last1[1], last2[1])
    assert last1[2:] == last2[2:] and tot1 == tot2


def test_frames_in_flight_sharded_frame_world1():
    """prt.tiles.ShardedFrame (the caller's torch.distributed gather) with 3 frames in flight: the tile render of a
    call may still be on an internal stream when torch queues the gather, so ShardedFrame joins it first
    (prt_finish); every accumulated frame equals the unsharded one."""
    import socket

    import torch
    import torch.distributed as dist
    import prt
    sd = scenes.multi_instance(scenes.config_small(50, 40))
    W, H, n = 96, 64, 4
    ref = prt.Context(0)
    c = prt.Context(0)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        gpu_scene(ref, sd, W, H)
        want = [ref.render(W, H, 4, 3, frame_index=2 * f)[:2] for f in range(n)]
        gpu_scene(c, sd, W, H)
        shard = prt.tiles.ShardedFrame(c, dist, W, H, 32, device="cuda")
        c.set_frames_in_flight(3)
        got = []
        for f in range(n):
            avg = torch.zeros((H * W, 4), dtype=torch.float32, device="cuda")
            rgb = torch.zeros(H * W, dtype=torch.int32, device="cuda")
            shard.render(4, 3, avg.data_ptr(), rgb.data_ptr(), frame_index=2 * f, stats=False)
            got.append((avg, rgb))
        torch.cuda.synchronize()
        for f, ((o, g), (a, r)) in enumerate(zip(got, want)):
            assert np.array_equal(o.cpu().numpy(), a), f
            assert np.array_equal(g.cpu().numpy().view(np.uint32), r), f
    finally:
        c.close()
        ref.close()
        dist.destroy_process_group()


def test_frames_in_flight_refused_on_local_group():
    import prt
    g = prt.Context(group=[0, 0], tile=16)
    try:
        with pytest.raises(prt.PrtError):
            g.set_frames_in_flight(2)
        g.set_frames_in_flight(1)
        with pytest.raises(prt.PrtError):
            g.set_frames_in_flight(0)
    finally:
        g.close()
