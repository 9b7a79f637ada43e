#!/usr/bin/env python3
"""Kernel timeline of one rank's share of the C4 frame (world N, rank r; default world 8, rank 0) with bench.py's
frames in flight: run under `rocprofv3 --kernel-trace --output-format csv`, then
`scripts/share_timeline.py --analyze <kernel_trace.csv> [frames]` prints, over the last `frames` frames, the wall
time per frame, the time some kernel is running (union), the sum of kernel durations (÷ union = mean concurrency)
and per kernel name the count and mean duration: what the share's frame is made of.

usage: share_timeline.py [world] [rank]          (env PRT_RANK_INFLIGHT as rank_time.py; PRT_TL_FRAMES: timed frames, 20)
       share_timeline.py --analyze <csv> [frames]"""
import os
import sys


def analyze(path, frames):
    import csv
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         r.get("Queue_Id", "")))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if "k_wave_init" in r[2]]
    if len(starts) < frames + 1:
        raise SystemExit(f"{len(starts)} frames in the trace, {frames} asked")
    first = starts[-frames]
    win = [r for r in rows[first:] if "k_" in r[2]]
    t0 = win[0][0]
    t1 = max(r[1] for r in win)
    busy, cur_s, cur_e = 0, None, None
    for s, e, _, _ in win:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    total = sum(e - s for s, e, _, _ in win)
    print(f"{frames} frames: {(t1 - t0) / 1e6 / frames:.3f} ms per frame, some kernel running "
          f"{busy / (t1 - t0):.3f} of it, kernel time {total / 1e6 / frames:.3f} ms per frame "
          f"(mean concurrency {total / busy:.2f})")
    names = {}
    for s, e, n, q in win:
        k = n.split("(")[0].replace("void ", "")
        names.setdefault(k, []).append(e - s)
    for k, d in sorted(names.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {k:60s} {len(d) / frames:5.1f} per frame  mean {sum(d) / len(d) / 1e3:8.1f} us  "
              f"min {min(d) / 1e3:7.1f}  max {max(d) / 1e3:7.1f}  {sum(d) / 1e6 / frames:.3f} ms per frame")
    queues = {}
    for s, e, n, q in win:
        queues.setdefault(q, 0)
        queues[q] += e - s
    print("  per queue (ms per frame): " + ", ".join(f"{q}: {v / 1e6 / frames:.3f}" for q, v in sorted(queues.items())))


if len(sys.argv) > 1 and sys.argv[1] == "--analyze":
    analyze(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 20)
    sys.exit(0)

import time  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "physically-based-ray-tracer_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import prt  # noqa: E402
from prt import scenes  # noqa: E402
from bench import default_inflight  # noqa: E402

WORLD = int(sys.argv[1]) if len(sys.argv) > 1 else 8
RANK = int(sys.argv[2]) if len(sys.argv) > 2 else 0
INFLIGHT = int(os.environ.get("PRT_RANK_INFLIGHT", str(default_inflight(WORLD))))
C5 = os.environ.get("PRT_TL_SCENE", "c4") == "c5"  # PRT_TL_SCENE=c5: the C5 frame (3840x2160, 16 spp, depth 8)
W, H, SPP, BOUNCES, TILE = (3840, 2160, 16, 8, 32) if C5 else (1920, 1080, 4, 4, 32)
FPC = SPP // 2
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
# bench.py's order: RCCL first, then the context on its own stream with its flight streams
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
ctx = prt.Context(0)
ctx.set_stream(None)
sd = scenes.config_c5() if C5 else scenes.config_c4()
ctx.set_scene(prt.Scene.from_data(sd))
ctx.set_camera(prt.Camera(sd.cam_pos, sd.cam_target, np.float32(W) / np.float32(H)))
ctx.set_frames_in_flight(INFLIGHT)
per = ctx.tile_buffer_pixels(W, H, TILE, WORLD)
tiles = torch.zeros((per, 4), dtype=torch.float32, device="cuda")
torch.cuda.synchronize()


def frame(i):
    ctx.render_tiles(W, H, SPP, BOUNCES, TILE, RANK, WORLD, tiles.data_ptr(), frame_index=FPC * i)


k = 0
tw = time.perf_counter()
while time.perf_counter() - tw < 0.5:
    frame(k)
    k += 1
    if k % 4 == 0:
        torch.cuda.synchronize()
ctx.finish()
ctx.ray_totals(reset=True)
torch.cuda.synchronize()
NT = int(os.environ.get("PRT_TL_FRAMES", "20"))
t0 = time.perf_counter()
for i in range(NT):
    frame(k + i)
ctx.finish()
torch.cuda.synchronize()
ms = (time.perf_counter() - t0) * 1e3 / NT
seg, sh = ctx.ray_totals(reset=True)
print(f"world {WORLD} rank {RANK}: {INFLIGHT} in flight, {ms:.3f} ms per frame over the last {NT} frames, "
      f"{(seg + sh) // NT} rays per frame", flush=True)
ctx.close()
dist.destroy_process_group()
