#!/usr/bin/env python3
"""Strong-scaling estimate of the pixel-tile sharding on ONE GPU: every rank's share of the
C4 (or C5) frame for world = 2, 4, 8, each share warmed alone, plus the per-frame collective work rank 0 adds.

For each world N and rank r = 0..N-1: PRT_RANK_WARM_S seconds of that rank's own share frames (the GPU's clock
state follows the load), then n timed frames -> ms(r).  An N-GPU frame is gated by the slowest rank, so
    frame(N) = max_r ms(r)                                  (collectives overlapped by the frames in flight)
    frame(N, serial) = max_r ms(r) + gather + untile        (no overlap at all: an upper bound)
gather = a world-1 RCCL ncclGather (torch.distributed "nccl" over this one GPU) of rank 0's tile buffer
(W*H*16/N bytes), untile = prt_untile of the N gathered buffers into the W x H image; both timed with HIP
events over 50 repetitions.  Efficiency = ms(world 1) / (N * frame(N)), against world 1 one frame at a time and
with the same frames in flight.

usage: rank_time.py [c5] [worlds...]   (env PRT_RANK_INFLIGHT: frames in flight of the shares; default bench.py's)
prints one line per (world, rank) and a summary line per world; the timed frames run without stats, as bench.py's."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "physically-based-ray-tracer_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import prt  # noqa: E402
from prt import scenes  # noqa: E402

args = sys.argv[1:]
sys.path.insert(0, ROOT)
from bench import default_inflight  # noqa: E402
# frames in flight of the shares (default: bench.py's on several GPUs) and of the world-1 frame (bench.py's on one)
INFLIGHT = int(os.environ.get("PRT_RANK_INFLIGHT", str(default_inflight(8))))
INFLIGHT1 = default_inflight(1)
WARM_S = float(os.environ.get("PRT_RANK_WARM_S", "0.5"))
C5 = bool(args) and args[0] == "c5"
if C5:
    args = args[1:]
WORLDS = [int(a) for a in args] or [2, 4, 8]
sd = scenes.config_c5() if C5 else scenes.config_c4()
W, H, SPP, BOUNCES = (3840, 2160, 16, 8) if C5 else (1920, 1080, 4, 4)
FPC = SPP // 2
TILE = 32
# bench.py's order on several GPUs: RCCL first (torch.distributed; here world 1, for the gather timing), then the
# context on its own stream (torch's null stream maps to it) with its frames-in-flight streams created at once --
# HIP deals a process's streams over its hardware queues as they are created (profiles/r06_stream_ab.txt).
# PRT_RANK_STREAM=side puts the context on a torch side stream instead (A/B).  The untile is timed on a side stream
# either way, so that torch's events see it.
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29531")
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
ctx = prt.Context(0)
SIDE = os.environ.get("PRT_RANK_STREAM", "own") == "side"
side = torch.cuda.Stream() if SIDE else None
ctx.set_stream(side.cuda_stream if SIDE else None)
ctx.set_scene(prt.Scene.from_data(sd))
ctx.set_camera(prt.Camera(sd.cam_pos, sd.cam_target, np.float32(W) / np.float32(H)))
ctx.set_frames_in_flight(max(INFLIGHT, INFLIGHT1))
# timed frames per share (env PRT_RANK_FRAMES): 40 C4 frames (≈ 45 ms at world 8) -- with 8, one slow frame
# moved a rank's share by up to 10 % and the max over ranks with it
NT = int(os.environ.get("PRT_RANK_FRAMES", "4" if C5 else "40"))


def share_ms(world, rank, inflight):
    """rank's share of the frame (world 1: the whole frame), warmed alone, n frames timed back to back."""
    ctx.set_frames_in_flight(inflight)
    per = ctx.tile_buffer_pixels(W, H, TILE, world)
    tiles = torch.zeros((per, 4), dtype=torch.float32, device="cuda")
    avg = torch.zeros((H * W, 4), dtype=torch.float32, device="cuda")
    rgb = torch.zeros(H * W, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()  # (the buffers are filled on the null stream, the frames run on the context's stream)

    def frame(i):
        if world == 1:
            ctx.render(W, H, SPP, BOUNCES, frame_index=FPC * i, avg=avg.data_ptr(), rgb8=rgb.data_ptr(),
                       device_out=True, stats=False)
        else:
            ctx.render_tiles(W, H, SPP, BOUNCES, TILE, rank, world, tiles.data_ptr(), frame_index=FPC * i)
    frame(0)
    torch.cuda.synchronize()
    tw = time.perf_counter()
    k = 1
    while time.perf_counter() - tw < WARM_S:
        frame(k)
        k += 1
        if k % 4 == 0:
            torch.cuda.synchronize()
    ctx.finish()
    ctx.ray_totals(reset=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(NT):
        frame(i)
    ctx.finish()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / NT
    seg, sh = ctx.ray_totals(reset=True)
    return ms, (seg + sh) // NT


def event_ms(fn, on, reps=50):
    """mean ms of fn over reps, HIP events on stream `on` (the stream fn's work runs on)"""
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(on)
    for _ in range(reps):
        fn()
    b.record(on)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def collective_ms(world):
    """world-1 RCCL gather of rank 0's tile buffer + prt_untile of world gathered buffers (rank 0's extra work)."""
    per = ctx.tile_buffer_pixels(W, H, TILE, world)
    part = torch.zeros((per, 4), dtype=torch.float32, device="cuda")
    bufs = [torch.zeros_like(part)]
    g = event_ms(lambda: dist.gather(part, bufs, dst=0), torch.cuda.current_stream())  # (torch's RCCL ordering)
    gathered = torch.zeros((world * per, 4), dtype=torch.float32, device="cuda")
    avg = torch.zeros((H * W, 4), dtype=torch.float32, device="cuda")
    rgb = torch.zeros(H * W, dtype=torch.int32, device="cuda")
    ctx.finish()
    torch.cuda.synchronize()
    us = side or torch.cuda.Stream()
    ctx.set_stream(us.cuda_stream)
    u = event_ms(lambda: ctx.untile(gathered.data_ptr(), W, H, TILE, world, avg.data_ptr(), rgb.data_ptr()), us)
    ctx.set_stream(side.cuda_stream if SIDE else None)
    return g, u, per * 16


scene = "c5" if C5 else "c4"
w1_one, rays1 = share_ms(1, 0, 1)
w1_fl, _ = share_ms(1, 0, INFLIGHT1)
print(f"{scene} world 1: frame {w1_one:.3f} ms one at a time, {w1_fl:.3f} ms with {INFLIGHT1} in flight  rays {rays1}; "
      f"shares below with {INFLIGHT} in flight", flush=True)
for world in WORLDS:
    ms = []
    for r in range(world):
        m, rays = share_ms(world, r, INFLIGHT)
        ms.append(m)
        print(f"  world {world} rank {r}: share {m:.3f} ms  rays {rays}", flush=True)
    g, u, nbytes = collective_ms(world)
    mx = max(ms)
    ser = mx + g + u
    print(f"{scene} world {world}: max share {mx:.3f} ms (rank {int(np.argmax(ms))}), mean {np.mean(ms):.3f}, "
          f"min {min(ms):.3f}; gather {g:.3f} ms ({nbytes / 1e6:.2f} MB, world-1 RCCL) + untile {u:.3f} ms; "
          f"efficiency vs {INFLIGHT1}-in-flight world 1: {w1_fl / (world * mx):.3f} overlapped, "
          f"{w1_fl / (world * ser):.3f} serial; vs one-at-a-time world 1: {w1_one / (world * mx):.3f} / "
          f"{w1_one / (world * ser):.3f}", flush=True)
ctx.close()
dist.destroy_process_group()
