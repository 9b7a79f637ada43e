#!/usr/bin/env python3
"""Summarise one scripts/gpu_mem.sh session (gpurun_out/mem_<tag>_<scene>) into profiles/<tag>_<scene>_mem.json:
per kernel, the mean per dispatch of every counter of every pass, and the derived vector-memory figures that say
which stage of the memory path bounds it:

- ta_busy / td_busy: TA_TA_BUSY_sum / TD_TD_BUSY_sum over (256 CUs x the kernel's cycles), the cycles are
  GRBM_GUI_ACTIVE / 8 XCDs of the same pass (each TA / TD is one per CU);
- td_tc_stall: TD_TC_STALL_sum over the same CU-cycles (the data return waiting on the cache);
- tcp_pending_stall: TCP_PENDING_STALL_CYCLES_sum over the CU-cycles (L1 out of miss slots);
- l2_read_latency_cycles: TCP_TCC_READ_REQ_LATENCY_sum / TCP_TCC_READ_REQ_sum (mean L1 -> L2 read round trip);
- l1_hit_rate: 1 - TCP_TCC_READ_REQ_sum / TCP_TOTAL_CACHE_ACCESSES_sum; l2_hit_rate: TCC_HIT / (TCC_HIT + TCC_MISS);
- vmem_per_wave, salu_per_wave etc. from the SQ pass (SQ_WAVES from the launch grid is not counted here: waves =
  SQ_WAVE_CYCLES / mean wave cycles is not available, so per-launch totals are reported).
usage: scripts/summarize_mem.py <tag> <scene> [session dir]"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "physically-based-ray-tracer_amd"))
from prt import codeobj  # noqa: E402

NCU, NXCD = 256, 8


def short(name):
    return name.split("(")[0].replace("void ", "").strip().split("::")[-1].split("<")[0]


def pass_means(path):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    return {k: {c: v / len(disp[k]) for c, v in d.items()} for k, d in per.items()}, {k: len(v) for k, v in disp.items()}


def main():
    tag, scene = sys.argv[1], sys.argv[2]
    src = sys.argv[3] if len(sys.argv) > 3 else os.path.join(ROOT, "gpurun_out", f"mem_{tag}_{scene}")
    out = {"name": f"{tag}_{scene}_mem", "scene": scene,
           "command": f"python3 bench.py --scene {scene} --no-cpu-baseline --steps 1 --warmup 1 --inflight 1 "
                      "(scripts/gpu_mem.sh, one rocprofv3 --pmc pass per counter group)",
           "passes": {}, "kernels": {}}
    K = out["kernels"]
    for p in sorted(os.listdir(src)):
        f = os.path.join(src, p, "run_counter_collection.csv")
        if not os.path.isfile(f):
            continue
        means, calls = pass_means(f)
        out["passes"][p] = sorted({c for d in means.values() for c in d})
        for k, d in means.items():
            r = K.setdefault(k, {"counters": {}, "cycles": {}})
            for c, v in d.items():
                if c == "GRBM_GUI_ACTIVE":
                    r["cycles"][p] = v / NXCD
                else:
                    r["counters"][c] = v
    hashes = {}
    hf = os.path.join(src, "lib_hashes.json")
    if os.path.exists(hf):
        hashes = json.load(open(hf)).get("kernels", {})
    for k, r in K.items():
        c, cyc = r["counters"], r["cycles"]

        def frac(counter, pas):
            if counter in c and cyc.get(pas):
                return round(c[counter] / (NCU * cyc[pas]), 4)
            return None
        d = {"ta_busy": frac("TA_TA_BUSY_sum", "ta"), "td_busy": frac("TD_TD_BUSY_sum", "td"),
             "td_tc_stall": frac("TD_TC_STALL_sum", "td"),
             "ta_addr_stalled_by_tc": frac("TA_ADDR_STALLED_BY_TC_CYCLES_sum", "ta2"),
             "ta_data_stalled_by_tc": frac("TA_DATA_STALLED_BY_TC_CYCLES_sum", "ta2"),
             "tcp_pending_stall": frac("TCP_PENDING_STALL_CYCLES_sum", "tcp"),
             "tcp_ta_data_stall": frac("TCP_TCP_TA_DATA_STALL_CYCLES_sum", "tcp"),
             "tcp_tcr_stall": frac("TCP_TCR_TCP_STALL_CYCLES_sum", "tcp2"),
             "tcp_tagconflict_stall": frac("TCP_READ_TAGCONFLICT_STALL_CYCLES_sum", "tcp2")}
        if c.get("TCP_TCC_READ_REQ_sum"):
            d["l2_read_latency_cycles"] = round(c.get("TCP_TCC_READ_REQ_LATENCY_sum", 0) / c["TCP_TCC_READ_REQ_sum"], 1)
            if c.get("TCP_TOTAL_CACHE_ACCESSES_sum"):
                d["l1_hit_rate"] = round(1 - c["TCP_TCC_READ_REQ_sum"] / c["TCP_TOTAL_CACHE_ACCESSES_sum"], 4)
        if c.get("TCC_HIT_sum") is not None and c.get("TCC_MISS_sum") is not None:
            d["l2_hit_rate"] = round(c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"]), 4)
        if c.get("SQ_INSTS_VMEM_RD"):
            d["tcp_accesses_per_vmem_rd"] = round(c.get("TCP_TOTAL_CACHE_ACCESSES_sum", 0) / c["SQ_INSTS_VMEM_RD"], 2)
            d["valu_per_vmem_rd"] = round(c.get("SQ_INSTS_VALU", 0) / c["SQ_INSTS_VMEM_RD"], 2)
            if cyc.get("sq"):
                d["ta_cycles_per_vmem_rd"] = round(c.get("TA_TA_BUSY_sum", 0) / c["SQ_INSTS_VMEM_RD"], 2)
        if c.get("SQ_WAVE_CYCLES"):
            d["wait_frac"] = round(c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"], 4)
        r["derived"] = {a: b for a, b in d.items() if b is not None}
        kh = {h: v for h, v in hashes.items() if short(h) == k or h == k}
        if kh:
            r["code_hash"] = next(iter(kh.values()))
    path = os.path.join(ROOT, "profiles", f"{tag}_{scene}_mem.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    with open(os.path.join(ROOT, "profiles", f"current_{scene}_mem.json"), "w") as f:  # what bench.py reads
        json.dump(out, f, indent=1)
    for k in ("k_trace2", "k_shade2", "k_res2d"):
        if k in K:
            print(k, json.dumps(K[k]["derived"]))
    print("wrote", path)


if __name__ == "__main__":
    main()
