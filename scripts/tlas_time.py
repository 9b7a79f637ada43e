#!/usr/bin/env python3
"""Per-frame instance BVH update (the reference's BVH::Build over its BLASInstances every frame,
Core/Renderer.cpp:33-41): N moving tori over the heightfield (scenes.instance_field), every instance moved before
every frame, frames queued back to back.  Device refit of the instance BVH (default, prt_tlas.hip) against a host
SAH rebuild + upload per frame (PRT_TLAS_HOST=1): ms per frame and the host time of prt_set_instances."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "physically-based-ray-tracer_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import prt  # noqa: E402
from prt import scenes  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
sd = scenes.instance_field(N, seed=3)
W, H = 1280, 720
ctx = prt.Context(0)
ctx.set_stream(torch.cuda.current_stream().cuda_stream)
ctx.set_scene(prt.Scene.from_data(sd))
ctx.set_camera(prt.Camera(sd.cam_pos, sd.cam_target, np.float32(W) / np.float32(H)))
avg = torch.zeros((H * W, 4), dtype=torch.float32, device="cuda")
rgb = torch.zeros(H * W, dtype=torch.int32, device="cuda")
base = [(m, np.array(T, np.float32)) for m, T in sd.instances]
n = 20
for host in ("0", "1", "0", "1"):
    os.environ["PRT_TLAS_HOST"] = host
    for i in range(2):
        ctx.render(W, H, 2, 3, frame_index=i, avg=avg.data_ptr(), rgb8=rgb.data_ptr(), device_out=True, stats=False)
    torch.cuda.synchronize()
    upd = 0.0
    t0 = time.perf_counter()
    for i in range(n):
        inst = []
        for k, (m, T) in enumerate(base):
            T = T.copy()
            if m == 1:
                T[0, 3] += np.float32(0.2 * np.sin(0.3 * i + k))
                T[2, 3] += np.float32(0.2 * np.cos(0.2 * i + k))
            inst.append((m, T))
        u0 = time.perf_counter()
        ctx.set_instances(inst)
        upd += time.perf_counter() - u0
        ctx.render(W, H, 2, 3, frame_index=i, avg=avg.data_ptr(), rgb8=rgb.data_ptr(), device_out=True, stats=False)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) * 1e3 / n
    print(f"{N} instances, {'host rebuild' if host == '1' else 'device refit'}: {dt:.3f} ms/frame, "
          f"prt_set_instances {upd * 1e6 / n:.1f} us host, tlas depth {ctx.scene_info().tlas_depth}", flush=True)
ctx.close()
