#!/usr/bin/env python3
"""Child processes of tests/test_gpu_bench_config.py (each run in a fresh process, so that environment settings
that HIP or RCCL read once -- GPU_MAX_HW_QUEUES, PRT_RCCL_TIMEOUT_S -- apply from the first HIP call on).
Prints one JSON line.

  shard_child.py bench <frames_in_flight> <W> <H>
      bench.py's configuration on several GPUs, on this one: a torch.distributed "nccl" group (world 1 here), the
      context sharded inside the boundary (prt.tiles.join_rccl -> prt_shard_init_rccl, one ncclGather per frame),
      the given frames in flight (4 = bench.py's default from 2 GPUs, whose chains run on cut grids), C4's
      1M-triangle scene at W x H, 4 spp, depth 4; 6 accumulating frames with device outputs and an instance update
      before frame 3.  Every frame is compared with an unsharded context rendering the same sequence one frame at
      a time: {"frames": 6, "mismatch": [...], "world": 1, "queues": ...}
  shard_child.py stall
      a world-2 communicator whose second rank never joins: prt_shard_init_rccl must fail within the time limit
      (PRT_RCCL_TIMEOUT_S) instead of hanging: {"error": "...", "seconds": s}"""
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "physically-based-ray-tracer_amd"))

import numpy as np  # noqa: E402


def bench(flights, W, H):
    import torch
    import torch.distributed as dist
    import prt
    from prt import scenes
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    sd = scenes.config_c4()
    moved = []
    for m, T in sd.instances:
        T = np.array(T, np.float32).copy()
        T[0, 3] += np.float32(0.031)
        T[2, 3] -= np.float32(0.017)
        moved.append((m, T))
    scene = prt.Scene.from_data(sd)
    cam = prt.Camera(sd.cam_pos, sd.cam_target, np.float32(W) / np.float32(H))

    def run(shard):
        c = prt.Context(0)
        side = torch.cuda.Stream()  # the context's stream, as bench.py sets it (outputs allocated in its order)
        try:
            c.set_stream(side.cuda_stream)
            c.set_scene(scene)
            c.set_camera(cam)
            world = 1
            if shard:
                c.set_frames_in_flight(flights)
                world = prt.tiles.join_rccl(c, dist, 32).world
            outs = []
            for f in range(6):
                if f == 3:
                    c.set_instances(moved)
                with torch.cuda.stream(side):
                    avg = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
                    rgb = torch.zeros(W * H, dtype=torch.int32, device="cuda")
                c.render(W, H, 4, 4, frame_index=2 * f, avg=avg.data_ptr(), rgb8=rgb.data_ptr(), device_out=True,
                         stats=False)
                outs.append((avg, rgb))
            c.finish()
            torch.cuda.synchronize()
            tot = c.ray_totals()
            return [(a.cpu().numpy(), r.cpu().numpy()) for a, r in outs], tot, world
        finally:
            c.close()
    ref, tref, _ = run(False)
    got, tgot, world = run(True)
    bad = [k for k, ((a1, r1), (a2, r2)) in enumerate(zip(ref, got))
           if not (np.array_equal(a1, a2) and np.array_equal(r1, r2))]
    dist.destroy_process_group()
    return {"frames": len(got), "mismatch": bad, "world": world, "totals_equal": tuple(tref) == tuple(tgot),
            "queues": os.environ.get("GPU_MAX_HW_QUEUES"), "flights": flights}


def stall():
    import prt
    c = prt.Context(0)
    t0 = time.perf_counter()
    err = None
    try:
        c.shard_rccl(prt.Context.shard_unique_id(), 0, 2, 32)  # rank 1 never comes
    except prt.PrtError as e:
        err = str(e)
    dt = time.perf_counter() - t0
    c.close()
    return {"error": err, "seconds": round(dt, 2)}


if __name__ == "__main__":
    mode = sys.argv[1]
    out = bench(int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])) if mode == "bench" else stall()
    print(json.dumps(out), flush=True)
