#!/usr/bin/env python3
"""bench.py -- BASELINE.json's metric: Mrays/s (+ ms/frame) at 1920x1080, 4 spp, depth 4.

Workload (config C4, the 1M-triangle scene the north-star target is quoted on; it fits one MI355X):
1000x500-quad heightfield = 1,000,000 triangles, procedural textures, 4 point + directional + spot
light, equirect sky, camera (0.3,3,-7) -> origin, all reference features on (AA, accumulate, gamma,
normal map, skybox, lighted, stochastic NEE).  A step = one prt_render of the full 4-spp frame
(2 reference frames x 2 AA paths per pixel), inputs resident in HBM.  Two frames are in flight by default
(prt_set_frames_in_flight): step k+1's wavefront chain overlaps step k's on the GPU, the accumulation (and the
sharded gather) stay in step order, and every step's image is bit-identical to rendering them one at a time; the
K timed steps are all complete when the closing synchronize returns.  Before them: the W warmup steps and, untimed
as well, as many more as fill --warmup-s (0.5 s) of frames, the same count on every rank (config.warmup_steps_run).

Mrays/s = (closest-hit segments + any-hit shadow rays) / time, counted on the device.
--gpus N > 1: one process per GPU.  Run without WORLD_SIZE in the environment, bench.py starts the N ranks
itself (torch.distributed.run as a child process, before anything touches a GPU) and exits with their
status.  Every rank's context joins one RCCL communicator inside the C ABI (prt_shard_init_rccl): each renders
its 32x32 pixel tiles (round-robin) and prt_render gathers the tile buffers on rank 0 with one ncclGather per
frame; value = all ranks' rays / max-over-ranks time.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "physically-based-ray-tracer_amd"))

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
# VALU issue peak: 256 CUs x 4 SIMD-32 x 2.4 GHz, one wave64 VALU instruction per 2 cycles per SIMD
# (MI355X_MICROARCH.md, Execution model) = 1228.8 G wave-instructions/s
VALU_PEAK_GINST = 256 * 4 * 2.4 / 2  # G wave64 VALU instructions/s: 1024 SIMDs x 2.4 GHz / 2 cycles each
VISITS_JSON = os.path.join(ROOT, "profiles", "reference_visits_c4.json")
TRACE_KERNEL = "k_trace2"


def algorithmic_bytes_per_ray():
    """B_ray = 256*N_int + 192*N_leaf + 64*N_tlas + 192*N_inst + 48 + 16, with N measured on the
    reference's own BVH8_CPU (tinybvh v1.4.2, oracle/_ref) for this workload (profiles/reference_visits_c4.json)."""
    with open(VISITS_JSON) as f:
        v = json.load(f)
    out = {}
    for kind in ("closest", "anyhit"):
        n = v[kind]
        out[kind] = 256.0 * n["n_int"] + 192.0 * n["n_leaf"] + 64.0 * n["n_tlas"] + 192.0 * n["n_inst"] + 48 + 16
    return out


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


def _pmc_kernel(path, kernel):
    """Per-launch record of `kernel` in a committed profile summary (scripts/summarize_prof.py)."""
    if not os.path.exists(path):
        return None, None
    with open(path) as fh:
        t = json.load(fh)
    for name, d in t.get("kernels", {}).items():
        if name.split("::")[-1].split("<")[0] == kernel:
            return d, t.get("name")
    return None, None


def current_code_hash(kernel):
    """Hash of `kernel`'s machine code in the libprt.so being timed (prt/codeobj.py: the gfx950 code objects
    of the library's .hip_fatbin, the kernel's .text bytes + kernel descriptor, all instantiations)."""
    from prt import _lib, codeobj
    try:
        return codeobj.base_hashes(_lib.LIBPATH).get(kernel)
    except (OSError, ValueError):
        return None


def fresh(d, live_hash):
    """A committed PMC record prices the timed library only when it carries the same code hash."""
    return bool(d) and live_hash is not None and d.get("code_hash") == live_hash


def profile_record(scene, kernel):
    """Per-launch record of `kernel` in profiles/current_<scene>.json (scripts/gpu_prof.sh + summarize_session.py:
    rocprofv3 --stats, FETCH_SIZE / WRITE_SIZE, VALU-issue and stall --pmc passes of `bench.py --scene <scene>`,
    stamped with the code hash of the kernels they measured)."""
    return _pmc_kernel(os.path.join(ROOT, "profiles", f"current_{scene}.json"), kernel)


def memory_record(scene, kernel):
    """Derived vector-memory figures of `kernel` in profiles/current_<scene>_mem.json (scripts/gpu_mem.sh +
    summarize_mem.py: TA / TD / TCP / TCC / SQ passes of `bench.py --scene <scene>`), with its code hash."""
    path = os.path.join(ROOT, "profiles", f"current_{scene}_mem.json")
    if not os.path.exists(path):
        return None, None
    with open(path) as fh:
        t = json.load(fh)
    d = t.get("kernels", {}).get(kernel)
    return d, t.get("name")


def host_cpu():
    """CPU model, logical CPUs of the host, and the CPUs this process may use (affinity / cgroup quota)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    usable = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()
            if q != "max":
                usable = min(usable, max(1, int(int(q) // int(p))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit():
        usable = min(usable, int(omp))
    return model, os.cpu_count() or 1, usable


def cpu_baseline(sd, W, H, spp, bounces):
    """Two CPU legs on a bounded sample of the same workload, timed on this host's cores (rank 0, N=1):
    'port'       -- the oracle: the C restatement of Renderer::Trace + its own traversal (OpenMP over rows);
    'reference'  -- the same restated Trace running on the reference's own tinybvh BVH8_CPU + TLAS traversal
                    (oracle/_ref, compiled from /root/reference/Core/tiny_bvh.h), the reference renderer's
                    hot path minus the shading code that cannot be compiled here.
    Sample: the full frame when it is <= ~300M rays-bounces, else a centred camera crop with the same spp /
    depth (pixels are independent, so Mrays/s carries over).  The reference leg's BVH8_CPU build is outside
    the timed region, like the GPU's BLAS build."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    model, nproc, threads = host_cpu()
    scale = 1
    while W * H * spp * bounces // (scale * scale) > 300_000_000:
        scale *= 2
    w, h = W // scale, H // scale
    what = "the full frame" if scale == 1 else f"the same camera at {w}x{h} (1/{scale * scale} of the pixels)"
    legs = []
    osc = oracle.OracleScene(sd, w, h)

    def timed(nthreads):
        t0 = time.perf_counter()
        _, _, _, st = osc.render(w, h, spp=spp, bounces=bounces, nthreads=nthreads)
        dt = time.perf_counter() - t0
        rays = st.segments + st.shadow_rays
        return {"value": round(rays / dt / 1e6, 2), "unit": "Mrays/s", "seconds": round(dt, 3), "rays": int(rays),
                "threads": nthreads}

    legs.append(dict(kind="port", **timed(threads)))
    ref_ok = oracle.reflib() is not None
    if ref_ok:
        osc.use_reference_traversal()
        points = [timed(t) for t in sorted({1, min(4, threads), threads})]
        legs.append(dict(kind="reference", **points[-1]))
    else:
        legs.append({"kind": "reference", "value": None, "why": "oracle/_ref/libref_tinybvh.so not built"})
        points = []
    ref = legs[1] if legs[1].get("value") else legs[0]
    out = {"value": ref["value"], "unit": "Mrays/s", "cores": threads, "kind": ref["kind"],
           "model": model, "host_logical_cpus": nproc,
           "sample": f"{sd.name}: {what}, {spp} spp, depth {bounces}, {threads} threads "
                     f"(this GPU's CPU share of a {nproc}-CPU host)",
           "legs": legs}
    if len(points) >= 2:  # measured only: the reference leg at 1, 4 and all usable threads of this GPU's CPU share
        out["thread_points"] = [{"threads": p["threads"], "value": p["value"], "seconds": p["seconds"]} for p in points]
    return out


def default_inflight(gpus):
    """Frames in flight bench.py keeps by default (prt_set_frames_in_flight; profiles/r06_rank_shares.txt): 2 on one
    GPU, 4 on several (each chain on a third or half of the resident blocks)."""
    return 4 if gpus >= 2 else 2


def spawn_ranks(n):
    """--gpus N without WORLD_SIZE: start N ranks of this script under torch.distributed.run (a child process;
    nothing here has touched a GPU) and return their exit status."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


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
    ap.add_argument("--context-stream", default="own", choices=["own", "side"],
                    help="the context's HIP stream: its own (default; torch's null stream maps to it) or a torch side "
                         "stream (A/B, profiles/r06_stream_ab.txt)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--inflight", type=int, default=None, choices=range(1, 9),
                    help="frames in flight (prt_set_frames_in_flight; default 2 on one GPU, 4 on several): "
                         "consecutive frames' wavefront chains overlap on internal streams; accumulation and "
                         "gathers stay in call order, the images are bit-identical to 1")
    ap.add_argument("--warmup-s", type=float, default=0.5,
                    help="untimed warmup of at least this many seconds of frames besides the W steps (the same step "
                         "count on every rank): a few milliseconds of frames leave the GPU below its clocks")
    ap.add_argument("--hw-queues", type=int, default=None,
                    help="opt-in: GPU_MAX_HW_QUEUES for this process (set before HIP starts); default: the runtime's "
                         "own setting (4 on the GPU box), which is what the library's users get")
    ap.add_argument("--host-out", action="store_true",
                    help="outputs (avg + rgb8) to host memory every step: the PCIe-inclusive rate (not the contract value)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    # Frames in flight: the best measured setting per share size (profiles/r05_inflight.txt): 2 for the whole
    # frame, 4 (with cut grids per chain) for the shares of 2-8 GPUs.  Each chain runs on its own HIP stream, and
    # HIP maps a process's streams onto GPU_MAX_HW_QUEUES hardware queues (4 by default) round-robin.  The headline
    # runs on the runtime's own queue count; --hw-queues is an explicit opt-in (set before anything initialises
    # HIP), and at world 8 the 4-queue share measured the faster one (profiles/r06_rank_shares_inflight_queues.txt)
    if args.inflight is None:
        args.inflight = default_inflight(args.gpus)
    if args.hw_queues:
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)

    import torch
    import prt
    from prt import scenes

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    dist = None
    dev = torch.device("cuda", local)
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    sd = {"c3": scenes.config_c3, "c4": scenes.config_c4, "c5": scenes.config_c5}[args.scene]()
    big = args.scene == "c5"
    args.width = args.width or (3840 if big else 1920)
    args.height = args.height or (2160 if big else 1080)
    args.spp = args.spp or (16 if big else 4)
    args.bounces = args.bounces if args.bounces is not None else (8 if big else 4)
    W, H = args.width, args.height
    ctx = prt.Context(local)
    # torch's current stream is the null stream here, so the context runs on its own (non-blocking) stream; a torch
    # side stream measured 3,880-3,887 Mrays/s at N = 1 against 4,040 (the two frames in flight did not overlap;
    # profiles/r06_stream_ab.txt)
    cstream = torch.cuda.Stream(device=dev) if args.context_stream == "side" else None
    ctx.set_stream(cstream.cuda_stream if cstream is not None else torch.cuda.current_stream().cuda_stream)
    scene = prt.Scene.from_data(sd)
    ctx.set_scene(scene)
    ctx.set_camera(prt.Camera(sd.cam_pos, sd.cam_target, np.float32(W) / np.float32(H)))
    info = ctx.scene_info()
    ranks_seen = 1
    ctx.set_frames_in_flight(args.inflight)
    if world > 1:
        si = prt.tiles.join_rccl(ctx, dist, args.tile)
        one = torch.ones(1, dtype=torch.float32, device=dev)
        dist.all_reduce(one)  # the rank count over the torch RCCL group ...
        ranks_seen = int(one.item())
        if ranks_seen != world or si.world != world:  # ... and the context's own communicator
            raise SystemExit(f"rank {rank}: {ranks_seen} ranks in the torch group, {si.world} in the context")

    avg = torch.zeros((H * W, 4), dtype=torch.float32, device=dev)
    rgb = torch.zeros(H * W, dtype=torch.int32, device=dev)
    avg_h = np.zeros((H * W, 4), np.float32) if args.host_out else None
    rgb_h = np.zeros(H * W, np.uint32) if args.host_out else None
    fpc = max(1, args.spp // 2)  # reference frames per call (AA: 2 paths each): distinct RNG streams per step

    def step(i, stats):
        if args.host_out:
            _, _, st = ctx.render(W, H, args.spp, args.bounces, frame_index=fpc * i, avg=avg_h, rgb8=rgb_h,
                                  device_out=False, stats=stats)
        else:
            _, _, st = ctx.render(W, H, args.spp, args.bounces, frame_index=fpc * i, avg=avg.data_ptr(),
                                  rgb8=rgb.data_ptr(), device_out=True, stats=stats)
        return st

    # Warmup: the W steps asked for, then (untimed too) as many more as fill --warmup-s seconds at the rate the W
    # steps ran, the same count on every rank (the frames' gathers are collective).  Two frames are a few ms at
    # world 8, too short for the GPU to reach its clocks: C4's world-8 share measured 1.34-1.40 ms per frame cold
    # against 1.14-1.17 ms warm (profiles/r05_warmup.txt)
    torch.cuda.synchronize()
    n0 = max(1, args.warmup)  # (at least one step, to time the rate)
    tw = time.perf_counter()
    for i in range(n0):
        step(i, False)
    torch.cuda.synchronize()
    per = (time.perf_counter() - tw) / n0
    extra = int(min(2000, max(0.0, args.warmup_s - per * n0) / max(per, 1e-4))) if args.warmup_s > 0 else 0
    if dist:
        e = torch.tensor([extra], dtype=torch.int64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        extra = int(e.item())
    for i in range(n0, n0 + extra):
        step(i, False)
    warm_steps = n0 + extra
    ctx.ray_totals(reset=True)  # waits for the warmup frames
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    # The frames are enqueued back to back: rays are counted on the device (prt_ray_totals) and read once after
    # the timed region, so no frame waits for the host.  The last timed frame also carries the per-launch HIP
    # event timers of the traversal kernel (stats=True; its host wait coincides with the closing synchronize).
    t0 = time.perf_counter()
    for i in range(args.steps):
        st = step(warm_steps + i, i == args.steps - 1)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    seg, shadow = ctx.ray_totals()
    ms_closest = [st.ms_closest]
    iters = st.iterations
    seg_local, shadow_local = seg, shadow
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
        # Roofline of the dominant kernel (k_trace2: the merged closest + shadow traversal, one launch per
        # wavefront iteration), per launch.  Launch time: HIP events recorded on the render stream around every
        # launch of the last timed frame (stats.ms_closest sums them).  Counts per launch: rocprofv3 PMC passes of this same
        # command, committed under profiles/ (SQ_INSTS_VALU; FETCH_SIZE + WRITE_SIZE).
        launches = max(1, iters)
        kern_ms = max(float(np.mean(ms_closest)) / launches, 1e-9)  # (the stats frame carries the per-launch events)
        seg_f, sh_f = seg_local / args.steps, shadow_local / args.steps  # rank 0's rays: its launches
        # the PMC passes are of each scene's default configuration at N = 1 (scripts/gpu_prof.sh)
        default_cfg = {"c3": (1920, 1080, 4, 4), "c4": (1920, 1080, 4, 4), "c5": (3840, 2160, 16, 8)}[args.scene]
        priced = (W, H, args.spp, args.bounces) == default_cfg and world == 1
        rec, rec_src = profile_record(args.scene, TRACE_KERNEL) if priced else (None, None)
        # the committed counters count only if they were taken on this very k_trace2 (code-object hash):
        # otherwise frac is withheld and the line says the profile is stale
        live_hash = current_code_hash(TRACE_KERNEL)
        stale = bool(rec) and not fresh(rec, live_hash)
        ok = bool(rec) and not stale
        valu = rec if ok and "SQ_INSTS_VALU" in rec else None
        traffic = int(rec["hbm_bytes_per_launch"]) if ok and "hbm_bytes_per_launch" in rec else None
        stall = rec.get("stall") if ok else None
        mrec, mrec_src = memory_record(args.scene, TRACE_KERNEL) if priced else (None, None)
        mem = mrec.get("derived") if mrec and fresh(mrec, live_hash) else None
        valu_rate = valu["SQ_INSTS_VALU"] / (kern_ms / 1e3) / 1e9 if valu else None
        hbm_rate = traffic / (kern_ms / 1e3) / 1e9 if traffic else None
        bpr = algorithmic_bytes_per_ray()
        ref_bytes = (seg_f * bpr["closest"] + sh_f * bpr["anyhit"]) / launches
        own = own_layout_bytes_per_ray()
        own_bytes = (seg_f * own["closest"] + sh_f * own["anyhit"]) / launches if own else None
        hbm = {"achieved": round(hbm_rate, 1) if hbm_rate else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
               "frac": round(hbm_rate / HBM_PEAK_GBS, 4) if hbm_rate else None, "traffic": traffic,
               "source": rec_src}
        # what bounds the kernel, from its stall counters: waves parked on s_waitcnt (dependent loads) most of
        # their cycles = latency, otherwise the VALU issue rate; with no fresh stall pass nothing is claimed
        if not stall:
            bound = None
        elif stall["wait"] > stall["issuing"] + stall["issue_stall"]:
            # parked on s_waitcnt most of the time: with the memory pipeline's counters, the vector-memory path
            # (the L1's misses in flight: TD busy / TCP pending stalls) when its data unit is near saturation
            bound = "vector-memory" if mem and mem.get("td_busy", 0) >= 0.8 else "latency"
        else:
            bound = "valu"
        if valu_rate is not None:
            roof = {"bound": bound, "achieved": round(valu_rate, 1), "peak": VALU_PEAK_GINST,
                    "unit": "G VALU wave-instructions/s", "frac": round(valu_rate / VALU_PEAK_GINST, 4),
                    "traffic": traffic, "valu_insts_per_launch": int(valu["SQ_INSTS_VALU"]), "source": rec_src,
                    # the single-wave issue rate (4 cycles per wave64 instruction, MI355X_MICROARCH.md
                    # constants table) bounds a SIMD holding one wave; k_trace2 holds 7, so frac uses 2 cycles
                    "frac_vs_single_wave_issue": round(2 * valu_rate / VALU_PEAK_GINST, 4)}
            if "valu_busy" in valu:  # SQ_ACTIVE_INST_VALU x 4 / SIMD cycles: waves with a VALU instruction in
                # flight (a lone wave holds its SIMD 4 cycles per instruction), not the 2-cycle issue peak above
                roof["wave_valu_active_pmc"] = round(valu["valu_busy"], 4)
            if valu.get("clock_ghz"):  # effective clock of the PMC pass (GRBM_GUI_ACTIVE / 8 / dispatch time)
                roof["pmc_clock_ghz"] = round(valu["clock_ghz"], 3)
                roof["frac_at_pmc_clock"] = round(valu_rate / (VALU_PEAK_GINST * valu["clock_ghz"] / 2.4), 4)
        else:  # no fresh VALU pass for this config: price the measured HBM bytes (or nothing)
            roof = {"bound": bound, "achieved": hbm["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": hbm["frac"], "traffic": traffic}
        if mem:
            roof["memory"] = {k: mem[k] for k in ("ta_busy", "td_busy", "td_tc_stall", "tcp_pending_stall", "l1_hit_rate",
                                                 "l2_hit_rate", "l2_read_latency_cycles") if k in mem}
            roof["memory"]["source"] = mrec_src
        if stall:
            roof["stall"] = {k: round(v, 4) for k, v in stall.items()}
            roof["bound_basis"] = ("stall = fractions of SQ_WAVE_CYCLES: wait = parked on s_waitcnt (SQ_WAIT_ANY), "
                                   "issue_stall = SQ_WAIT_INST_ANY, issuing = SQ_ACTIVE_INST_ANY; bound = latency "
                                   "when wait > issuing + issue_stall, vector-memory when moreover the texture data "
                                   "unit is busy >= 0.8 of the kernel's cycles (memory.td_busy)")
        roof["stale_profile"] = stale
        roof["code_hash"] = live_hash[:16] if live_hash else None
        roof.update({
            "kernel": TRACE_KERNEL, "per": f"launch (avg of {launches} launches per frame)",
            "launch_ms": round(kern_ms, 4), "launch_timing": "HIP events around each launch of the last timed frame",
            "hbm": hbm,
            "algorithmic_bytes_per_launch": round(ref_bytes),
            # SURVEY 8d's per-ray bytes priced in the reference's BVH8_CPU layout (256-B nodes, 192-B leaves), as if
            # every visit came from HBM: above the HBM peak, so not an HBM figure (the tree sits in L2 / MALL)
            "reference_layout_equiv": {"GBps": round(ref_bytes / (kern_ms / 1e3) / 1e9, 1),
                                       "note": "not an HBM figure (SURVEY 8d reference-layout bytes / launch time; "
                                               "exceeds the 8 TB/s peak)"},
            "own_layout_equiv_GBps": round(own_bytes / (kern_ms / 1e3) / 1e9, 1) if own_bytes else None,
            "basis": "frac = PMC-measured VALU wave-instructions (SQ_INSTS_VALU) per second over the issue peak "
                     "(1024 SIMDs x 2.4 GHz / 2 cycles per wave64 instruction, MI355X_MICROARCH.md); "
                     "hbm = PMC-measured HBM bytes over the HBM peak; memory = the vector-memory path's busy / stall "
                     "fractions (scripts/gpu_mem.sh TA / TD / TCP / TCC passes)",
            "bytes_per_ray": {k: round(v, 1) for k, v in bpr.items()},
        })
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
            "ranks_seen": ranks_seen,
            "data": "synthetic (seeded procedural heightfield, textures, sky; scenes.py)",
            "config": {"workload": f"{sd.name}: {info.triangles} tris, {W}x{H}, {args.spp} spp, depth {args.bounces}",
                       "global_batch": W * H, "seq_len": args.bounces,
                       "parallelism": f"pixel-tile{args.tile} x{world} (RCCL gather in prt_render)" if world > 1
                       else "single-gpu",
                       "outputs": "host memory (PCIe-inclusive)" if args.host_out else "device (HBM-resident)",
                       "frames_in_flight": args.inflight, "warmup_steps_run": warm_steps,
                       "warmup_min_s": args.warmup_s,
                       "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "runtime default (4)"),
                       "rays_per_step": int(rays / args.steps), "segments_per_step": int(seg / args.steps),
                       "shadow_per_step": int(shadow / args.steps),
                       "mpix_per_s": round(W * H / (ms_step / 1e3) / 1e6, 2),
                       # camera paths (one Trace chain per camera ray: W*H*spp per frame) and the
                       # reference's own "Mrays/s" label, pixels per second (Core/Renderer.cpp:473)
                       "mpaths_per_s": round(W * H * args.spp / (ms_step / 1e3) / 1e6, 2),
                       "reference_style_mrays_per_s": round(W * H / (ms_step / 1e3) / 1e6, 2)},
            "roofline": roof,
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(sd, W, H, args.spp, args.bounces)
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
