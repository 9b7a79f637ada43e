#!/usr/bin/env python3
"""Summaries of the rocprofv3 --pmc passes behind bench.py's roofline (MI355X_MICROARCH.md, HBM / rocprofv3).

  valu <name> [dir]         gpurun_out/pmc_valu/run_counter_collection.csv (SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU,
                            SQ_WAVE_CYCLES, SQ_BUSY_CYCLES, SQ_WAVES, GRBM_GUI_ACTIVE) -> profiles/<name>.json: per-launch means per kernel, plus
                              valu_busy = SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)
                              (SQ_ACTIVE_INST_VALU counts quad-cycles; GRBM_GUI_ACTIVE is summed over the 8 XCDs)
  calib <name> [dir]        scripts/bin/fetch_calibration under FETCH_SIZE / WRITE_SIZE passes
                            (gpurun_out/calib_fetch, calib_write, calib_known.json) -> profiles/<name>.json:
                            known bytes / (counter KiB x 1024) per access shape = the correction factor
"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from summarize_prof import stamp  # noqa: E402


def short(name):
    return name.split("(")[0].replace("void ", "").strip()


def per_launch(path, durations=None):
    """{kernel: {counter: mean over dispatches of the per-dispatch sum}} and dispatch counts.  With a dict
    `durations`, also {kernel: mean dispatch ns} of this pass when the CSV carries timestamps."""
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    span = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
        if r.get("Start_Timestamp") and r.get("End_Timestamp"):
            span[k][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    if durations is not None:
        for k, d in span.items():
            durations[k] = sum(d.values()) / len(d)
    return {k: {c: v / len(disp[k]) for c, v in d.items()} for k, d in per.items()}, {k: len(v) for k, v in disp.items()}


def valu(name, src):
    dur = {}
    means, calls = per_launch(os.path.join(src, "pmc_valu", "run_counter_collection.csv"), dur)
    stats = {}  # fallback durations: the --kernel-trace --stats pass of the same session
    sf = os.path.join(src, "prof_stats", "run_kernel_stats.csv")
    if os.path.exists(sf):
        stats = {short(r["Name"]): float(r["AverageNs"]) for r in csv.DictReader(open(sf))}
    out = {"name": name, "source": "rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES "
                                   "SQ_WAVES GRBM_GUI_ACTIVE -- python3 bench.py --steps 1 --warmup 1", "kernels": {}}
    for k, d in means.items():
        if not k.startswith("prt::"):
            continue
        rec = dict(d)
        rec["calls"] = calls[k]
        if d.get("GRBM_GUI_ACTIVE"):
            rec["valu_busy"] = d.get("SQ_ACTIVE_INST_VALU", 0.0) * 4 / (1024 * d["GRBM_GUI_ACTIVE"] / 8)
            # effective shader clock of the pass (MI355X_MICROARCH.md, DVFS give-back: GRBM_GUI_ACTIVE / 8 XCDs
            # / dispatch wall time); the dispatch time is this pass's own when the CSV has timestamps
            ns, ns_src = (dur[k], "pmc pass timestamps") if k in dur else (stats.get(k), "kernel-trace stats")
            if ns:
                rec["dispatch_ns"] = ns
                rec["clock_ghz"] = d["GRBM_GUI_ACTIVE"] / 8 / ns
                rec["clock_source"] = ns_src
        out["kernels"][k] = rec
    stamp(out, src)
    for fn in (f"{name}.json",):  # bench.py prices profiles/current_<scene>.json (scripts/summarize_session.py)
        with open(os.path.join(ROOT, "profiles", fn), "w") as f:
            json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


def calib(name, src):
    known = json.load(open(os.path.join(src, "calib_known.json")))
    fetch, _ = per_launch(os.path.join(src, "calib_fetch", "run_counter_collection.csv"))
    write, _ = per_launch(os.path.join(src, "calib_write", "run_counter_collection.csv"))
    out = {"name": name, "program": "scripts/fetch_calibration.hip", "kernels": {}}
    for k, kb in known.items():
        f = next((v for n, v in fetch.items() if n.endswith(k)), {})
        w = next((v for n, v in write.items() if n.endswith(k)), {})
        rec = {"known_read_bytes": kb["read"], "known_write_bytes": kb["write"],
               "FETCH_SIZE_kib": f.get("FETCH_SIZE"), "WRITE_SIZE_kib": w.get("WRITE_SIZE")}
        if f.get("FETCH_SIZE"):
            rec["read_factor"] = kb["read"] / (f["FETCH_SIZE"] * 1024)
        if w.get("WRITE_SIZE"):
            rec["write_factor"] = kb["write"] / (w["WRITE_SIZE"] * 1024)
        out["kernels"][k] = rec
    with open(os.path.join(ROOT, "profiles", f"{name}.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    what, name = sys.argv[1], sys.argv[2]
    src = sys.argv[3] if len(sys.argv) > 3 else os.path.join(ROOT, "gpurun_out")
    {"valu": valu, "calib": calib}[what](name, src)
