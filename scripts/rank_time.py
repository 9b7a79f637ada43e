#!/usr/bin/env python3
"""Per-rank frame time of the pixel-tile sharding on ONE GPU: rank 0's share of the C4 frame for
world = 1, 2, 4, 8 (what each GPU of an N-GPU node renders), to estimate strong scaling without a node."""
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
W, H = 1920, 1080
ctx = prt.Context(0)
ctx.set_stream(torch.cuda.current_stream().cuda_stream)
ctx.set_scene(prt.Scene.from_data(sd))
ctx.set_camera(prt.Camera(sd.cam_pos, sd.cam_target, np.float32(W) / np.float32(H)))
base = None
WORLDS = [int(a) for a in sys.argv[1:]] or [1, 2, 4, 8]
for world in WORLDS:
    per = ctx.tile_buffer_pixels(W, H, 32, world)
    tiles = torch.zeros((per, 4), dtype=torch.float32, device="cuda")
    for i in range(2):
        ctx.render_tiles(W, H, 4, 4, 32, 0, world, tiles.data_ptr(), frame_index=2 * i)
    torch.cuda.synchronize()
    n = 5
    t0 = time.perf_counter()
    for i in range(n):
        st = ctx.render_tiles(W, H, 4, 4, 32, 0, world, tiles.data_ptr(), frame_index=2 * i, stats=True)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / n
    base = base or ms * world
    print(f"world {world}: rank-0 frame {ms:.3f} ms  rays {st.segments + st.shadow_rays}  "
          f"ideal {base / world:.3f} ms  efficiency {base / world / ms:.2f}", flush=True)
