#!/usr/bin/env python3
"""Which hardware queues a context's frames in flight land on (diagnostic; run under rocprofv3 --kernel-trace and
read with scripts/overlap.py): bench.py's N >= 2 sequence at world 1 -- torch.distributed (RCCL) initialised first,
the context on its own stream (or a torch side stream), N frames in flight, an RCCL communicator joined inside the
boundary (world 1) -- then C4 frames back to back.  usage: queue_probe.py <inflight> <own|side> [rccl|plain]"""
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "physically-based-ray-tracer_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import prt  # noqa: E402
from prt import scenes  # noqa: E402

fl, kind = int(sys.argv[1]), sys.argv[2]
rccl = len(sys.argv) < 4 or sys.argv[3] == "rccl"
if rccl:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
sd = scenes.config_c4()
W, H = 1920, 1080
ctx = prt.Context(0)
side = torch.cuda.Stream() if kind == "side" else None
ctx.set_stream(side.cuda_stream if side is not None else torch.cuda.current_stream().cuda_stream)
ctx.set_scene(prt.Scene.from_data(sd))
ctx.set_camera(prt.Camera(sd.cam_pos, sd.cam_target, np.float32(W) / np.float32(H)))
ctx.set_frames_in_flight(fl)
if rccl:
    prt.tiles.join_rccl(ctx, dist, 32)
avg = torch.zeros((H * W, 4), dtype=torch.float32, device="cuda")
rgb = torch.zeros(H * W, dtype=torch.int32, device="cuda")
torch.cuda.synchronize()
t0 = time.perf_counter()
n = 12
for i in range(n):
    ctx.render(W, H, 4, 4, frame_index=2 * i, avg=avg.data_ptr(), rgb8=rgb.data_ptr(), device_out=True, stats=False)
ctx.finish()
torch.cuda.synchronize()
print(f"{fl} in flight, {kind} stream, {'rccl' if rccl else 'plain'}: {(time.perf_counter() - t0) * 1e3 / n:.3f} ms per frame")
ctx.close()
if rccl:
    dist.destroy_process_group()
