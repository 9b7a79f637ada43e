#!/usr/bin/env python3
"""Per-dispatch timeline of the last frame in a rocprofv3 --kernel-trace CSV (k_wave_init .. k_accumulate).
usage: scripts/frame_timeline.py [gpurun_out/prof_stats/run_kernel_trace.csv]"""
import csv
import sys

f = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_stats/run_kernel_trace.csv"
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
s = [i for i, r in enumerate(rows) if "k_wave_init" in r["Kernel_Name"]][-1]
e = [i for i, r in enumerate(rows) if "k_accumulate" in r["Kernel_Name"] and i > s][0]
t0 = int(rows[s]["Start_Timestamp"])
busy = gaps = 0
prev = None
per = {}
for r in rows[s:e + 1]:
    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("void prt::", "").replace("prt::", "")[:28]
    gap = (st - prev) / 1e3 if prev else 0.0
    gaps += gap
    per[name.split("<")[0]] = per.get(name.split("<")[0], 0) + (en - st) / 1e3
    print(f"{name:28s} start {(st - t0) / 1e3:8.1f} dur {(en - st) / 1e3:7.1f} gap {gap:6.1f}")
    busy += en - st
    prev = en
print(f"frame {(prev - t0) / 1e3:.1f} us  busy {busy / 1e3:.1f}  gaps {gaps:.1f}")
print({k: round(v, 1) for k, v in per.items()})
