#!/usr/bin/env python3
"""Instance-BVH drift: N tori drift across the field for F frames (every instance moved
before every frame, wrapping at the field's edge; 1280x720, 2 spp, depth 3), under the library's policy
(prt_api.cpp ensure_instances: a host SAH build for every update, on the context's worker thread, the stream waiting
for each update's build before its upload).

The frames are paced as a render loop presenting them would: at most PACE (env PRT_DRIFT_PACE, default 3; 0: no
pacing, frames queued back to back) frames are queued when an update is made, the wait for the oldest outside the
timed call.  Reports: ms per frame over the drift; the host time inside prt_set_instances per update (mean, p99,
max); the rebuilds the context counted, the worker's last build (wall and CPU ms) and its median-split fallbacks;
ms per frame of static frames at the final positions, against a fresh context's tree built over those positions.
usage: tlas_drift.py [N] [F]"""
import collections
import dataclasses
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
F = int(sys.argv[2]) if len(sys.argv) > 2 else 200
sd = scenes.instance_field(N, seed=17)
W, H = 1280, 720
PACE = int(os.environ.get("PRT_DRIFT_PACE", "3"))
INFLIGHT = int(os.environ.get("PRT_DRIFT_INFLIGHT", "1"))  # frames in flight of both contexts
# the contexts' stream: a torch side stream, so the pacing events below are recorded in the frames' order (torch's
# current stream is the null stream here, and prt_set_stream(NULL) means the context's own stream)
STREAM = torch.cuda.Stream()
OWN = os.environ.get("PRT_DRIFT_STREAM", "side") == "own"  # A/B: the context's own stream (pacing then off)
if OWN:
    PACE = 0
rng = np.random.default_rng(3)
vel = rng.uniform(-0.08, 0.08, (len(sd.instances), 2)).astype(np.float32)


def drift(inst):
    """Every torus moves by its velocity in x and z, wrapping at the field's edge (numpy: a per-instance Python loop
    would take as long as the frame)."""
    mi, T = inst
    T = T.copy()
    mv = mi == 1
    for k, a in ((0, 0), (1, 2)):
        x = T[:, a, 3] + vel[:, k]
        x = np.where(x > 4.5, x - np.float32(9.0), np.where(x < -4.5, x + np.float32(9.0), x)).astype(np.float32)
        T[:, a, 3] = np.where(mv, x, T[:, a, 3])
    return mi, T


def set_instances(ctx, inst):  # the ABI call itself (prt_set_instances), without the list packing of Renderer
    mi, T = inst
    _lib.check(ctx.L.prt_set_instances(ctx.h, T.ctypes.data, mi.ctypes.data, len(mi)))


def context(inst):
    """a fresh context whose first instance BVH is built over `inst` (the scene's own instances)"""
    ctx = prt.Context(0)
    ctx.set_stream(None if OWN else STREAM.cuda_stream)
    mi, T = inst
    ctx.set_scene(prt.Scene.from_data(dataclasses.replace(sd, instances=[(int(m), T[k]) for k, m in enumerate(mi)])))
    ctx.set_camera(prt.Camera(sd.cam_pos, sd.cam_target, np.float32(W) / np.float32(H)))
    ctx.set_frames_in_flight(INFLIGHT)
    return ctx


def frames(ctx, avg, rgb, n, inst=None, host_ms=None):
    torch.cuda.synchronize()
    queued = collections.deque()
    t0 = time.perf_counter()
    for i in range(n):
        if inst is not None:
            inst = drift(inst)
            while PACE and len(queued) >= PACE:  # the render loop's present of the oldest queued frame
                queued.popleft().synchronize()
            h0 = time.perf_counter()
            set_instances(ctx, inst)
            host_ms.append((time.perf_counter() - h0) * 1e3)
        ctx.render(W, H, 2, 3, frame_index=i, avg=avg.data_ptr(), rgb8=rgb.data_ptr(), device_out=True, stats=False)
        if PACE:
            ev = torch.cuda.Event()
            ev.record(STREAM)
            queued.append(ev)
    ctx.finish()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / n, inst


avg = torch.zeros((H * W, 4), dtype=torch.float32, device="cuda")
rgb = torch.zeros(H * W, dtype=torch.int32, device="cuda")
inst0 = (np.array([m for m, _ in sd.instances], np.uint32), np.stack([np.array(T, np.float32) for _, T in sd.instances]))
ctx = context(inst0)
frames(ctx, avg, rgb, 10)  # warm
host = []
ms_drift, inst = frames(ctx, avg, rgb, F, inst0, host)
si = ctx.scene_info()
ms_end, _ = frames(ctx, avg, rgb, 20)
ctx.close()
ref = context(inst)
frames(ref, avg, rgb, 5)
ms_ref, _ = frames(ref, avg, rgb, 20)
ref.close()
print(f"{N} instances, {F} frames of drift ({'own' if OWN else 'side'} stream, pace {PACE}, {INFLIGHT} in flight; stacks for {si.max_depth} + "
      f"{si.tlas_depth} levels): {ms_drift:.3f} ms/frame; set_instances host "
      f"{np.mean(host):.3f} ms mean, {np.percentile(host, 99):.3f} p99, {np.max(host):.3f} max; {si.tlas_rebuilds} "
      f"rebuilds ({si.tlas_async} on the worker, {si.tlas_median} median-split), last worker build "
      f"{si.tlas_build_ms:.2f} ms ({si.tlas_build_cpu_ms:.2f} ms CPU); static at the end {ms_end:.3f} ms/frame vs "
      f"{ms_ref:.3f} on a fresh tree ({(ms_end / ms_ref - 1) * 100:+.1f} %); drift vs fresh static "
      f"{ms_drift / ms_ref:.3f}x", flush=True)
