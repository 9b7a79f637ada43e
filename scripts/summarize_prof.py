#!/usr/bin/env python3
"""Summarise a gpu_check.sh 'prof' run (rocprofv3 --kernel-trace --stats + separate FETCH_SIZE / WRITE_SIZE
--pmc passes) into profiles/<name>.json and profiles/<name>_kernel_stats.csv.

HBM traffic per launch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reports 1/2 of the bytes of 128-B requests (TCC_EA0_RDREQ x 64 B), so read bytes = 2 x 1024 x
FETCH_SIZE; WRITE_SIZE is taken as 1024 x WRITE_SIZE.  Infinity-Cache hits are counted as fabric reads.

usage: scripts/summarize_prof.py <name> [gpurun_out]
(Round 4: superseded by scripts/gpu_prof.sh + scripts/summarize_session.py, whose profiles/current_<scene>.json
bench.py prices; this summariser is kept for the older gpu_check.sh 'prof' layout.)
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "physically-based-ray-tracer_amd"))
from prt import codeobj  # noqa: E402


def stamp(out, src):
    """Stamp every kernel record with the hash of the machine code it measured (codeobj.base_hashes): from
    <src>/lib_hashes.json, written on the GPU box before the passes, else from the in-tree libprt.so."""
    f = os.path.join(src, "lib_hashes.json")
    if os.path.exists(f):
        hashes, origin = json.load(open(f))["kernels"], "lib_hashes.json written on the GPU box"
    else:
        hashes = codeobj.base_hashes(os.path.join(ROOT, "physically-based-ray-tracer_amd", "prt", "libprt.so"))
        origin = "in-tree libprt.so at summary time"
    out["code_hash_source"] = origin
    for k, d in out["kernels"].items():
        h = hashes.get(codeobj.profile_kernel_base(k))
        if h:
            d["code_hash"] = h


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "").strip()


def main():
    name = sys.argv[1]
    src = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out")
    out = {"name": name, "kernels": {}}
    stats = os.path.join(src, "prof_stats", "run_kernel_stats.csv")
    for r in csv.DictReader(open(stats)):
        out["kernels"][short(r["Name"])] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                            "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"]),
                                            "pct": float(r["Percentage"])}
    for kind, counter, scale in (("fetch", "FETCH_SIZE", 2 * 1024), ("write", "WRITE_SIZE", 1024)):
        f = os.path.join(src, f"prof_{kind}", "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        agg = {}
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = short(r["Kernel_Name"])
            agg.setdefault(k, {}).setdefault(r["Dispatch_Id"], 0.0)
            agg[k][r["Dispatch_Id"]] += float(r["Counter_Value"])
        # frames in the pass = dispatches of k_wave_init (once per frame): a kernel's launches per frame are its
        # dispatches over that count (round 3 divided by a fixed 3 and overstated k_trace2's bytes per frame 1.5x)
        frames = next((len(v) for k2, v in agg.items() if k2.endswith("k_wave_init")), None)
        for k, per in agg.items():
            vals = list(per.values())
            d = out["kernels"].setdefault(k, {})
            d[f"{counter}_raw_kib_per_launch"] = sum(vals) / len(vals)
            d[f"hbm_{kind}_bytes_per_launch"] = sum(vals) / len(vals) * scale
            if frames:
                d["launches_per_frame"] = len(vals) / frames
                d[f"hbm_{kind}_bytes_per_frame"] = sum(vals) * scale / frames
    for k, d in out["kernels"].items():
        if "hbm_fetch_bytes_per_launch" in d or "hbm_write_bytes_per_launch" in d:
            d["hbm_bytes_per_launch"] = d.get("hbm_fetch_bytes_per_launch", 0) + d.get("hbm_write_bytes_per_launch", 0)
            d["hbm_bytes_per_frame"] = d.get("hbm_fetch_bytes_per_frame", 0) + d.get("hbm_write_bytes_per_frame", 0)
    stamp(out, src)
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", f"{name}.json"), "w") as f:
        json.dump(out, f, indent=1)
    shutil.copy(stats, os.path.join(ROOT, "profiles", f"{name}_kernel_stats.csv"))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
