#!/usr/bin/env python3
"""Summarise one scripts/gpu_prof.sh session (gpurun_out/prof_<tag>_<scene>) into
profiles/<tag>_<scene>_prof.json, profiles/<tag>_<scene>_kernel_stats.csv and profiles/current_<scene>.json
(what bench.py prices for that scene).

Per kernel:
- calls / avg_ns / min_ns / max_ns: the --kernel-trace --stats pass;
- launches_per_frame: dispatches of the kernel / dispatches of k_wave_init (once per frame) in the same pass;
- hbm_*_bytes_per_launch: FETCH_SIZE x 2 x 1024 + WRITE_SIZE x 1024 (MI355X_MICROARCH.md HBM section, gfx950
  FETCH_SIZE correction; checked for this kernel's access shapes in profiles/fetch_calibration.json), each from its
  own pass; hbm_bytes_per_frame = per launch x launches_per_frame;
- SQ_INSTS_VALU etc. per launch; valu_busy = SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8);
  clock_ghz = GRBM_GUI_ACTIVE / 8 XCDs / dispatch ns;
- stall fractions of SQ_WAVE_CYCLES: wait (SQ_WAIT_ANY: parked on s_waitcnt / barrier), issue_stall
  (SQ_WAIT_INST_ANY), issuing (SQ_ACTIVE_INST_ANY), valu (SQ_ACTIVE_INST_VALU);
- code_hash: the kernel's machine code in the library the session ran (lib_hashes.json, prt/codeobj.py).
usage: scripts/summarize_session.py <tag> <scene> [session dir]"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "physically-based-ray-tracer_amd"))
from prt import codeobj  # noqa: E402


def short(name):
    return name.split("(")[0].replace("void ", "").strip()


def pass_means(path):
    """{kernel: {counter: mean over dispatches of the per-dispatch sum}}, {kernel: dispatches}, {kernel: mean ns}"""
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    span = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
        if r.get("Start_Timestamp") and r.get("End_Timestamp"):
            span[k][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    means = {k: {c: v / len(disp[k]) for c, v in d.items()} for k, d in per.items()}
    ns = {k: sum(d.values()) / len(d) for k, d in span.items() if d}
    return means, {k: len(v) for k, v in disp.items()}, ns


def main():
    tag, scene = sys.argv[1], sys.argv[2]
    src = sys.argv[3] if len(sys.argv) > 3 else os.path.join(ROOT, "gpurun_out", f"prof_{tag}_{scene}")
    out = {"name": f"{tag}_{scene}", "scene": scene,
           "command": f"python3 bench.py --scene {scene} --no-cpu-baseline (scripts/gpu_prof.sh)", "kernels": {}}
    K = out["kernels"]
    stats = os.path.join(src, "stats", "run_kernel_stats.csv")
    for r in csv.DictReader(open(stats)):
        K[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]), "min_ns": float(r["MinNs"]),
                               "max_ns": float(r["MaxNs"]), "pct": float(r["Percentage"])}
    for kind, counter, scale in (("fetch", "FETCH_SIZE", 2 * 1024), ("write", "WRITE_SIZE", 1024)):
        f = os.path.join(src, kind, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        means, calls, _ = pass_means(f)
        init = next((n for k2, n in calls.items() if k2.endswith("k_wave_init")), None)
        for k, d in means.items():
            r = K.setdefault(k, {})
            r[f"{counter}_raw_kib_per_launch"] = d[counter]
            r[f"hbm_{kind}_bytes_per_launch"] = d[counter] * scale
            if init:
                r["launches_per_frame"] = calls[k] / init
    for k, r in K.items():
        if "hbm_fetch_bytes_per_launch" in r or "hbm_write_bytes_per_launch" in r:
            r["hbm_bytes_per_launch"] = r.get("hbm_fetch_bytes_per_launch", 0) + r.get("hbm_write_bytes_per_launch", 0)
            if "launches_per_frame" in r:
                r["hbm_bytes_per_frame"] = r["hbm_bytes_per_launch"] * r["launches_per_frame"]
    f = os.path.join(src, "valu", "run_counter_collection.csv")
    if os.path.exists(f):
        means, calls, ns = pass_means(f)
        for k, d in means.items():
            r = K.setdefault(k, {})
            r.update({c: v for c, v in d.items()})
            if d.get("GRBM_GUI_ACTIVE"):
                r["valu_busy"] = d.get("SQ_ACTIVE_INST_VALU", 0.0) * 4 / (1024 * d["GRBM_GUI_ACTIVE"] / 8)
                t = ns.get(k) or r.get("avg_ns")
                if t:
                    r["clock_ghz"] = d["GRBM_GUI_ACTIVE"] / 8 / t
    f = os.path.join(src, "stall", "run_counter_collection.csv")
    if os.path.exists(f):
        means, _, _ = pass_means(f)
        for k, d in means.items():
            wc = d.get("SQ_WAVE_CYCLES") or 0.0
            if wc <= 0:
                continue
            K.setdefault(k, {})["stall"] = {
                "wait": d.get("SQ_WAIT_ANY", 0.0) / wc, "issue_stall": d.get("SQ_WAIT_INST_ANY", 0.0) / wc,
                "issuing": d.get("SQ_ACTIVE_INST_ANY", 0.0) / wc, "valu": d.get("SQ_ACTIVE_INST_VALU", 0.0) / wc,
                "lds": d.get("SQ_ACTIVE_INST_LDS", 0.0) / wc, "scalar": d.get("SQ_ACTIVE_INST_SCA", 0.0) / wc}
    hf = os.path.join(src, "lib_hashes.json")
    hashes = json.load(open(hf))["kernels"] if os.path.exists(hf) else {}
    out["code_hash_source"] = "lib_hashes.json written on the GPU box before the passes" if hashes else "none"
    for k, r in K.items():
        h = hashes.get(codeobj.profile_kernel_base(k))
        if h:
            r["code_hash"] = h
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    for fn in (f"{tag}_{scene}_prof.json", f"current_{scene}.json"):
        with open(os.path.join(ROOT, "profiles", fn), "w") as fh:
            json.dump(out, fh, indent=1)
    shutil.copy(stats, os.path.join(ROOT, "profiles", f"{tag}_{scene}_kernel_stats.csv"))
    for k, r in K.items():
        if k.startswith("prt::"):
            print(k, {x: (round(v, 4) if isinstance(v, float) else v) for x, v in r.items() if not isinstance(v, dict)},
                  r.get("stall"))


if __name__ == "__main__":
    main()
