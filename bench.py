#!/usr/bin/env python3
"""bench.py -- BASELINE.json's metric: Mrays/s (+ ms/frame) at 1920x1080, 4 spp, depth 4.

Workload (config C4, the 1M-triangle scene the north-star target is quoted on; it fits one MI355X):
1000x500-quad heightfield = 1,000,000 triangles, procedural textures, 4 point + directional + spot
light, equirect sky, camera (0.3,3,-7) -> origin, all reference features on (AA, accumulate, gamma,
normal map, skybox, lighted, stochastic NEE).  A step = one prt_render of the full 4-spp frame
(2 reference frames x 2 AA paths per pixel), inputs resident in HBM.

Mrays/s = (closest-hit segments + any-hit shadow rays) / time, counted on the device.
N > 1: one process per GPU (torchrun), pixel tiles 32x32 round-robin over ranks, RCCL gather of the
per-rank tile buffers to rank 0, untile there; value = all ranks' rays / max-over-ranks time.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "physically-based-ray-tracer_amd"))

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
VISITS_JSON = os.path.join(ROOT, "profiles", "reference_visits_c4.json")


def algorithmic_bytes_per_ray():
    """B_ray = 256*N_int + 192*N_leaf + 64*N_tlas + 192*N_inst + 48 + 16, with N measured on the
    reference's own BVH8_CPU (tinybvh v1.4.2, oracle/_ref) for this workload (profiles/reference_visits_c4.json)."""
    with open(VISITS_JSON) as f:
        v = json.load(f)
    out = {}
    for kind in ("closest", "anyhit"):
        n = v[kind]
        out[kind] = 256.0 * n["n_int"] + 192.0 * n["n_leaf"] + 64.0 * n["n_tlas"] + 192.0 * n["n_inst"] + 48 + 16
    out["per_shaded_hit"] = 12.0   # 3 texels
    out["per_pixel_frame"] = 36.0  # accumulator read+write + rgb8
    return out, v


def own_layout_bytes_per_ray():
    """The build's own Node8 layout priced with its own visit counts (profiles/node8_visits_c4.json, from
    scripts/measure_node8_visits.py): 80 B per node visit + 48 B per triangle test + ray in / result out."""
    f = os.path.join(ROOT, "profiles", "node8_visits_c4.json")
    if not os.path.exists(f):
        return None
    with open(f) as fh:
        v = json.load(fh)
    c, a = v["all_closest"], v["all_anyhit"]
    return {"closest": v["node_bytes"] * c["node_visits"] + v["tri_bytes"] * c["tri_tests"] + 4 + 32 + 16,
            "anyhit": v["node_bytes"] * a["node_visits"] + v["tri_bytes"] * a["tri_tests"] + 32 + 1}


def measured_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes (profiles/traffic_current.json,
    written by scripts/summarize_prof.py; FETCH_SIZE x2 gfx950 correction, MI355X_MICROARCH.md HBM)."""
    f = os.path.join(ROOT, "profiles", "traffic_current.json")
    if not os.path.exists(f):
        return None
    with open(f) as fh:
        t = json.load(fh)
    for name, d in t.get("kernels", {}).items():
        base = name.split("::")[-1].split("<")[0]
        if base in (kernel, kernel + "_p", kernel + "2") and "hbm_bytes_per_launch" in d:
            return int(d["hbm_bytes_per_launch"])
    return None


def cpu_baseline(sd, threads, W, H, spp, bounces):
    """The oracle (C restatement, OpenMP over rows) on a bounded sample of the same workload: the full frame
    when it is <= ~40M rays (C4: ~29M rays, 10-30 s of CPU-core work), else a centred crop of the camera's
    pixel grid with the same spp / depth (every pixel-frame is independent, so Mrays/s carries over)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    scale = 1
    while W * H * spp * bounces // (scale * scale) > 300_000_000:
        scale *= 2
    w, h = W // scale, H // scale
    osc = oracle.OracleScene(sd, w, h)
    t0 = time.perf_counter()
    _, _, _, st = osc.render(w, h, spp=spp, bounces=bounces, nthreads=threads)
    dt = time.perf_counter() - t0
    rays = st.segments + st.shadow_rays
    what = "the full frame" if scale == 1 else f"the same camera at {w}x{h} (1/{scale * scale} of the pixels)"
    return {"value": rays / dt / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"{sd.name}: {what}, {spp} spp, depth {bounces} ({rays} rays, {dt:.2f} s)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--width", type=int, default=None, help="default 1920 (c3/c4), 3840 (c5)")
    ap.add_argument("--height", type=int, default=None, help="default 1080 (c3/c4), 2160 (c5)")
    ap.add_argument("--spp", type=int, default=None, help="default 4 (c3/c4), 16 (c5)")
    ap.add_argument("--bounces", type=int, default=None, help="default 4 (c3/c4), 8 (c5)")
    ap.add_argument("--scene", default="c4", choices=["c3", "c4", "c5"],
                    help="c4 = the metric's workload (default); c5 = C4 + a quad area light with MIS at 4K, 16 spp, depth 8")
    ap.add_argument("--tile", type=int, default=32)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--host-out", action="store_true",
                    help="outputs (avg + rgb8) to host memory every step: the PCIe-inclusive rate (not the contract value)")
    args = ap.parse_args()

    import torch
    import prt
    from prt import scenes

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)

    sd = {"c3": scenes.config_c3, "c4": scenes.config_c4, "c5": scenes.config_c5}[args.scene]()
    big = args.scene == "c5"
    args.width = args.width or (3840 if big else 1920)
    args.height = args.height or (2160 if big else 1080)
    args.spp = args.spp or (16 if big else 4)
    args.bounces = args.bounces if args.bounces is not None else (8 if big else 4)
    W, H = args.width, args.height
    ctx = prt.Context(local)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    scene = prt.Scene.from_data(sd)
    ctx.set_scene(scene)
    ctx.set_camera(prt.Camera(sd.cam_pos, sd.cam_target, np.float32(W) / np.float32(H)))
    info = ctx.scene_info()

    dev = torch.device("cuda", local)
    avg = torch.zeros((H * W, 4), dtype=torch.float32, device=dev)
    rgb = torch.zeros(H * W, dtype=torch.int32, device=dev)
    if world > 1:
        shard = prt.tiles.ShardedFrame(ctx, dist, W, H, args.tile, device=dev)

    avg_h = np.zeros((H * W, 4), np.float32) if args.host_out else None
    rgb_h = np.zeros(H * W, np.uint32) if args.host_out else None

    fpc = max(1, args.spp // 2)  # reference frames per call (AA: 2 paths each): distinct RNG streams per step

    def step(i):
        if world == 1 and args.host_out:
            _, _, st = ctx.render(W, H, args.spp, args.bounces, frame_index=fpc * i, avg=avg_h, rgb8=rgb_h,
                                  device_out=False, stats=True)
        elif world == 1:
            _, _, st = ctx.render(W, H, args.spp, args.bounces, frame_index=fpc * i, avg=avg.data_ptr(),
                                  rgb8=rgb.data_ptr(), device_out=True, stats=True)
        else:
            st = shard.render(args.spp, args.bounces, avg.data_ptr(), rgb.data_ptr(), frame_index=fpc * i)
        return st

    for i in range(args.warmup):
        step(i)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    seg = shadow = 0
    ms_trace, ms_closest, ms_anyhit = [], [], []
    pipeline = iters = batches = 0
    t0 = time.perf_counter()
    for i in range(args.steps):
        st = step(args.warmup + i)
        seg += st.segments
        shadow += st.shadow_rays
        ms_trace.append(st.ms_trace)
        ms_closest.append(st.ms_closest)
        ms_anyhit.append(st.ms_anyhit)
        pipeline = st.pipeline
        iters = st.iterations
        batches = st.batches
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    rays = seg + shadow
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        r = torch.tensor([seg, shadow], dtype=torch.float64, device=dev)
        dist.all_reduce(r)
        seg, shadow = int(r[0].item()), int(r[1].item())
        rays = seg + shadow

    if rank == 0:
        ms_step = elapsed * 1000.0 / args.steps
        value = rays / elapsed / 1e6
        bpr, visits = algorithmic_bytes_per_ray()
        # roofline of the dominant kernel, per launch: algorithmic bytes (reference BVH8_CPU visit counts x
        # SURVEY 8d bytes) of the rays one launch processes over the kernel's average launch duration (HIP events
        # recorded on the render stream around every launch; ms_closest / ms_anyhit sum them per frame)
        seg_f, sh_f = seg / args.steps, shadow / args.steps
        launches = max(1, iters) if pipeline in (0, 2) else 1
        kern = {}
        if pipeline == 2:  # merged pipeline: one traversal launch per iteration (closest + shadow rays)
            kern["k_trace"] = ((seg_f * bpr["closest"] + sh_f * bpr["anyhit"]) / launches,
                               float(np.mean(ms_closest)) / launches)
        elif pipeline == 3:  # streaming engine: one persistent launch per frame (traversal + shading)
            kern["k_stream"] = (seg_f * bpr["closest"] + sh_f * bpr["anyhit"], float(np.mean(ms_closest)))
        elif pipeline == 0:
            kern["k_extend"] = (seg_f * bpr["closest"] / launches, float(np.mean(ms_closest)) / launches)
            kern["k_shadow"] = (sh_f * bpr["anyhit"] / launches, float(np.mean(ms_anyhit)) / launches)
        else:
            kern["k_trace_frames"] = (seg_f * bpr["closest"] + sh_f * bpr["anyhit"], float(np.mean(ms_trace)))
        dom = max(kern, key=lambda k: kern[k][1])
        alg_bytes, kern_ms = kern[dom]
        kern_ms = max(kern_ms, 1e-9)  # PRT_LAUNCH_TIMERS=0 (A/B runs): no per-launch times
        achieved = alg_bytes / (kern_ms / 1e3) / 1e9
        traffic = measured_traffic(dom) if args.scene == "c4" else None  # the committed PMC passes are of C4
        own = own_layout_bytes_per_ray()
        own_block = None
        if own is not None and pipeline in (0, 2, 3):
            own_b = ((seg_f * own["closest"] if dom in ("k_extend", "k_trace", "k_stream") else 0.0) +
                     (sh_f * own["anyhit"] if dom in ("k_shadow", "k_trace", "k_stream") else 0.0)) / launches
            own_block = {"bytes_per_ray": {k: round(v, 1) for k, v in own.items()}, "algorithmic_bytes": round(own_b),
                         "achieved": round(own_b / (kern_ms / 1e3) / 1e9, 1),
                         "frac": round(own_b / (kern_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)}
        out = {
            "metric": f"Mrays/s (closest-hit segments + shadow any-hit rays) at {W}x{H}, {args.spp} spp, depth {args.bounces}",
            "value": round(value, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "strong",  # one fixed frame is split into pixel tiles over the N GPUs
            "vs_baseline": None,
            "dtype": "f32",
            "pipeline": {0: "wavefront", 1: "megakernel", 2: "wavefront-merged", 3: "stream"}[pipeline],
            "batches": batches,
            "data": "synthetic (seeded procedural heightfield, textures, sky; scenes.py)",
            "config": {"workload": f"{sd.name}: {info.triangles} tris, {W}x{H}, {args.spp} spp, depth {args.bounces}",
                       "global_batch": W * H, "seq_len": args.bounces,
                       "parallelism": f"pixel-tile{args.tile} x{world}" if world > 1 else "single-gpu",
                       "outputs": "host memory (PCIe-inclusive)" if args.host_out else "device (HBM-resident)",
                       "rays_per_step": int(rays / args.steps), "segments_per_step": int(seg / args.steps),
                       "shadow_per_step": int(shadow / args.steps),
                       "mpix_per_s": round(W * H / (ms_step / 1e3) / 1e6, 2),
                       # camera paths (one Trace chain per camera ray: W*H*spp per frame) and the
                       # reference's own "Mrays/s" label, pixels per second (Core/Renderer.cpp:473)
                       "mpaths_per_s": round(W * H * args.spp / (ms_step / 1e3) / 1e6, 2),
                       "reference_style_mrays_per_s": round(W * H / (ms_step / 1e3) / 1e6, 2)},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel": dom, "per": f"launch (avg of {launches} launches per frame)",
                         "basis": "SURVEY 8d algorithmic bytes in the reference's BVH8_CPU layout (256-B nodes, "
                                  "192-B leaves) -- frac > 1 means the same traversal in this build's 80-B Node8 / "
                                  "48-B triangle layout, served largely from L2 / Infinity Cache; own_layout prices "
                                  "this build's bytes, traffic is PMC-measured HBM",
                         "launch_ms": round(kern_ms, 4), "algorithmic_bytes": round(alg_bytes),
                         "kernels": {k: {"launch_ms": round(v[1], 4), "alg_GBps": round(v[0] / (v[1] / 1e3) / 1e9, 1)
                                         if v[1] > 0 else None} for k, v in kern.items()},
                         "bytes_per_ray": {k: round(v, 1) for k, v in bpr.items()},
                         "own_layout": own_block,
                         "traffic_GBps": round(traffic / (kern_ms / 1e3) / 1e9, 1) if traffic else None},
        }
        if world == 1 and not args.no_cpu_baseline:
            threads = min(16, os.cpu_count() or 1)
            out["cpu_baseline"] = cpu_baseline(sd, threads, W, H, args.spp, args.bounces)
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
