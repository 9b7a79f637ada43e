#!/usr/bin/env python3
"""Frame interval of the C4 frame (world 1) and of a world-8 share on different context streams (diagnostic):
the context's own stream (prt_set_stream(NULL)), a torch side stream, and the legacy null stream's torch current
stream as passed by bench.py (which maps to the own stream).  usage: stream_probe.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "physically-based-ray-tracer_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import prt  # noqa: E402
from prt import scenes  # noqa: E402

sd = scenes.config_c4()
W, H, SPP, B = 1920, 1080, 4, 4


def run(kind, fl, world, n=24):
    ctx = prt.Context(0)
    side = torch.cuda.Stream() if kind == "side" else None
    if side is not None:
        ctx.set_stream(side.cuda_stream)
    ctx.set_scene(prt.Scene.from_data(sd))
    ctx.set_camera(prt.Camera(sd.cam_pos, sd.cam_target, np.float32(W) / np.float32(H)))
    ctx.set_frames_in_flight(fl)
    avg = torch.zeros((H * W, 4), dtype=torch.float32, device="cuda")
    rgb = torch.zeros(H * W, dtype=torch.int32, device="cuda")
    per = ctx.tile_buffer_pixels(W, H, 32, world)
    tiles = torch.zeros((per, 4), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()

    def frame(i):
        if world == 1:
            ctx.render(W, H, SPP, B, frame_index=2 * i, avg=avg.data_ptr(), rgb8=rgb.data_ptr(), device_out=True,
                       stats=False)
        else:
            ctx.render_tiles(W, H, SPP, B, 32, 0, world, tiles.data_ptr(), frame_index=2 * i)
    t0 = time.perf_counter()
    k = 0
    while time.perf_counter() - t0 < 0.5:
        frame(k)
        k += 1
        if k % 4 == 0:
            ctx.finish()
            torch.cuda.synchronize()
    ctx.finish()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        frame(i)
    ctx.finish()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / n
    ctx.close()
    print(f"{kind:5s} stream, world {world}, {fl} in flight: {ms:.3f} ms per frame", flush=True)


for rep in range(2):
    for world, fl in ((1, 2), (8, 4)):
        for kind in ("own", "side"):
            run(kind, fl, world)
