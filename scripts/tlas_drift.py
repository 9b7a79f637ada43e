#!/usr/bin/env python3
"""Instance-BVH drift: N tori drift across the field for F frames (every instance moved before
every frame, wrapping at the field's edge; frames queued back to back, 1280x720, 2 spp, depth 3).  Per rebuild
policy: ms per frame over the drift, the host time spent inside set_instances per frame, then ms per frame of
static frames at the final positions against a fresh host SAH tree over the same positions (PRT_TLAS_HOST=1).
Modes (TLAS_MODES): unset = refit only / the default (up to 4,096 instances: the host SAH build for every update) /
the single-workgroup device build for every update / the multi-launch builder on the node-area trigger and every
frame; default / device / host = one of them once (host: a synchronous host SAH build per update)."""
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
rng = np.random.default_rng(3)
vel = rng.uniform(-0.08, 0.08, (len(sd.instances), 2)).astype(np.float32)
vel *= np.float32(os.environ.get("DRIFT_VEL", "1"))  # DRIFT_VEL=0: every instance re-set in place (the update machinery alone)


def drift(inst):
    """Every torus moves by its velocity in x and z, wrapping at the field's edge.  inst = (mesh ids uint32,
    transforms float32 [N,4,4]), updated in numpy (a per-instance Python loop took 3-4 ms a frame, close to the
    frame itself: the drift numbers would measure Python)."""
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


HOST_MS = []  # host time inside set_instances, per call


def timed(ctx, avg, rgb, n, inst=None):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        if inst is not None:
            inst = drift(inst)
            h0 = time.perf_counter()
            set_instances(ctx, inst)
            HOST_MS.append((time.perf_counter() - h0) * 1e3)
        ctx.render(W, H, 2, 3, frame_index=i, avg=avg.data_ptr(), rgb8=rgb.data_ptr(), device_out=True, stats=False)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / n, inst


MODES = [("refit only", "0", None), ("default (host SAH build, every update)", None, None),
         ("single-workgroup device build, every frame", None, "S"),
         ("multi-launch builder, trigger", "1.05", "M"), ("multi-launch builder, every frame", "always", "M")]
if os.environ.get("TLAS_MODES") == "trbvh":  # A/B of the device tree's treelet-restructuring passes
    MODES = [(f"device rebuild every frame, {k} TRBVH passes", "always", k) for k in ("0", "1", "2", "3")]
if os.environ.get("TLAS_MODES") == "radius":  # A/B of the device tree's PLOC radius (0 / 1 TRBVH passes)
    MODES = [(f"device rebuild every frame, PLOC radius {r}, {k} TRBVH passes", "always", k + ":" + r)
             for r, k in (("64", "0"), ("512", "0"), ("512", "1"))]
if os.environ.get("TLAS_MODES") == "small":  # the single-workgroup builder's policies
    MODES = [("small builder, trigger", "1.05", None), ("small builder, every frame", "always", None)]
if os.environ.get("TLAS_MODES") == "default":  # the default policy only, once (timeline sessions)
    MODES = MODES[1:2]
if os.environ.get("TLAS_MODES") == "device":  # the single-workgroup device build only, once
    MODES = MODES[2:3]
if os.environ.get("TLAS_MODES") == "host":  # a host SAH build for every update (the host waits; timeline sessions)
    MODES = [("host SAH build, every frame", None, "H")]
for mode, env, trbvh in MODES + (MODES if os.environ.get("TLAS_MODES") not in ("default", "host", "device") else []):
    os.environ.pop("PRT_TLAS_SMALL", None)
    host_every = trbvh == "H"
    if host_every:
        trbvh = None
    if trbvh == "S":  # the single-workgroup device build
        os.environ["PRT_TLAS_SMALL"] = "1"
        trbvh = "keep"
    if trbvh == "M":  # the multi-launch builder
        os.environ["PRT_TLAS_SMALL"] = "0"
        trbvh = None
    if trbvh in (None, "keep"):
        os.environ.pop("PRT_TLAS_TRBVH", None)
        os.environ.pop("PRT_TLAS_PLOC_R", None)
    else:  # (the treelet / radius knobs are the multi-launch builder's)
        os.environ["PRT_TLAS_SMALL"] = "0"
        os.environ["PRT_TLAS_TRBVH"] = trbvh.split(":")[0]
        if ":" in trbvh:
            os.environ["PRT_TLAS_PLOC_R"] = trbvh.split(":")[1]
    os.environ.pop("PRT_TLAS_HOST", None)
    if host_every:
        os.environ["PRT_TLAS_HOST"] = "1"
    if env is None:
        os.environ.pop("PRT_TLAS_REBUILD", None)
    else:
        os.environ["PRT_TLAS_REBUILD"] = env
    ctx = prt.Context(0)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    ctx.set_scene(prt.Scene.from_data(sd))
    ctx.set_camera(prt.Camera(sd.cam_pos, sd.cam_target, np.float32(W) / np.float32(H)))
    avg = torch.zeros((H * W, 4), dtype=torch.float32, device="cuda")
    rgb = torch.zeros(H * W, dtype=torch.int32, device="cuda")
    inst = (np.ascontiguousarray([m for m, _ in sd.instances], np.uint32),
            np.ascontiguousarray(np.stack([np.asarray(T, np.float32) for _, T in sd.instances])))
    timed(ctx, avg, rgb, 2)
    t_first, _ = timed(ctx, avg, rgb, 10)
    blocks = []
    HOST_MS.clear()
    for b in range(F // 20):
        ms, inst = timed(ctx, avg, rgb, 20, inst)
        blocks.append(round(ms, 3))
    si = ctx.scene_info()
    t_end, _ = timed(ctx, avg, rgb, 20)
    os.environ["PRT_TLAS_HOST"] = "1"
    set_instances(ctx, inst)  # a fresh host SAH tree over the final positions
    os.environ.pop("PRT_TLAS_HOST")
    os.environ["PRT_TLAS_REBUILD"] = "0"
    os.environ.pop("PRT_TLAS_SMALL", None)
    t_fresh, _ = timed(ctx, avg, rgb, 20)
    hd = ctx.scene_info().tlas_depth
    hms = np.array(HOST_MS)
    print(f"{N} instances, {F} frames, {mode}: static frame at start {t_first:.3f} ms; drift ms/frame per 20 frames "
          f"{blocks}; set_instances host time median {np.median(hms):.3f} / max {hms.max():.3f} ms; "
          f"{si.tlas_rebuilds} rebuilds ({si.tlas_rejected} device builds not committed) / {si.tlas_refits} refits; static frame at the end "
          f"{t_end:.3f} ms vs fresh host SAH tree {t_fresh:.3f} ms (depth {hd}) ({100 * (t_end / t_fresh - 1):+.1f} %)",
          flush=True)
    ctx.close()
