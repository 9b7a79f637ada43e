#!/usr/bin/env python3
"""Where prt_set_instances spends host time (diagnostic): N drifting tori, mean host time of the update call (and of
the render call) in three regimes -- updates only, update + render back to back, update + render + synchronize --
at 1 and 2 frames in flight, on three kinds of context stream (torch's current = the null stream, the context's
own, a torch side stream).  usage: inst_update_probe.py [N]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "physically-based-ray-tracer_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import prt  # noqa: E402
from prt import _lib, scenes  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
sd = scenes.instance_field(N, seed=17)
W, H = 1280, 720
mi = np.array([m for m, _ in sd.instances], np.uint32)
T0 = np.stack([np.array(T, np.float32) for _, T in sd.instances])


def run(fl, mode, kind, n=40):
    ctx = prt.Context(0)
    side = None
    if kind == "null":
        ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    elif kind == "side":
        side = torch.cuda.Stream()
        ctx.set_stream(side.cuda_stream)
    ctx.set_scene(prt.Scene.from_data(sd))
    ctx.set_camera(prt.Camera(sd.cam_pos, sd.cam_target, np.float32(W) / np.float32(H)))
    ctx.set_frames_in_flight(fl)
    avg = torch.zeros((H * W, 4), dtype=torch.float32, device="cuda")
    rgb = torch.zeros(H * W, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    T = T0.copy()
    up, rd = [], []
    for i in range(n):
        T[:, 0, 3] += np.where(mi == 1, np.float32(0.001), np.float32(0.0))
        h0 = time.perf_counter()
        _lib.check(ctx.L.prt_set_instances(ctx.h, T.ctypes.data, mi.ctypes.data, len(mi)))
        h1 = time.perf_counter()
        if mode != "updates":
            ctx.render(W, H, 2, 3, frame_index=i, avg=avg.data_ptr(), rgb8=rgb.data_ptr(), device_out=True, stats=False)
        h2 = time.perf_counter()
        if mode == "sync":
            ctx.finish()
            torch.cuda.synchronize()
        if i >= 5:
            up.append((h1 - h0) * 1e3)
            rd.append((h2 - h1) * 1e3)
    ctx.finish()
    torch.cuda.synchronize()
    ctx.close()
    print(f"N={N} {kind:5s} stream, in flight {fl} {mode:8s}: set_instances {np.mean(up):.3f} ms mean {np.max(up):.3f} max; "
          f"render call {np.mean(rd):.3f} ms mean", flush=True)


for kind in ("null", "own", "side"):
    for fl in (1, 2):
        for mode in ("sync", "queued"):
            run(fl, mode, kind)
