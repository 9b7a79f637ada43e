#!/usr/bin/env python3
"""Probe for frames in flight: rank 0's share of the C4 frame (world = 1 / 8, as rank_time.py) rendered by ONE
context frame after frame, against K contexts on the same GPU, each with its own stream, whose frames are
enqueued round-robin with no host wait -- K independent frame chains in flight at once.  Prints ms per frame for
each K: what a library that keeps K frames in flight could gain (no accumulation ordering between the contexts;
an upper bound for the real thing)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "physically-based-ray-tracer_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import prt  # noqa: E402
from prt import scenes  # noqa: E402

args = [int(a) for a in sys.argv[1:]]
WORLDS = args or [1, 8]
sd = scenes.config_c4()
W, H, SPP, BOUNCES = 1920, 1080, 4, 4
FPC = SPP // 2
scene = prt.Scene.from_data(sd)
cam = prt.Camera(sd.cam_pos, sd.cam_target, np.float32(W) / np.float32(H))
ctxs, streams = [], []
for k in range(3):
    s = torch.cuda.Stream()
    c = prt.Context(0)
    c.set_stream(s.cuda_stream)
    c.set_scene(scene)
    c.set_camera(cam)
    ctxs.append(c)
    streams.append(s)
for world in WORLDS:
    per = ctxs[0].tile_buffer_pixels(W, H, 32, world)
    tiles = [torch.zeros((per, 4), dtype=torch.float32, device="cuda") for _ in ctxs]
    for K in (1, 2, 3, 1, 2, 3):
        for k in range(K):
            ctxs[k].render_tiles(W, H, SPP, BOUNCES, 32, 0, world, tiles[k].data_ptr(), frame_index=0)
        torch.cuda.synchronize()
        n = 12 if world > 1 else 6
        t0 = time.perf_counter()
        for i in range(n):
            for k in range(K):
                ctxs[k].render_tiles(W, H, SPP, BOUNCES, 32, 0, world, tiles[k].data_ptr(), frame_index=FPC * i)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / (n * K)
        print(f"world {world}: {K} chain(s) in flight: {ms:.3f} ms per frame", flush=True)
for c in ctxs:
    c.close()
