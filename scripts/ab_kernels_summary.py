#!/usr/bin/env python3
"""One line per rocprofv3 --stats run (scripts/ab_kernels.sh): the variant, each kernel's mean duration (us) and
its total per frame (calls / k_wave_init calls), and the sum of kernel time per frame (ms).
usage: ab_kernels_summary.py <variant> <rocprofv3 output dir>"""
import csv
import glob
import sys

v, d = sys.argv[1], sys.argv[2]
f = glob.glob(f"{d}/**/run_kernel_stats.csv", recursive=True)[0]
rows = {}
for r in csv.DictReader(open(f)):
    k = r["Name"].split("(")[0].replace("void ", "").split("::")[-1].split("<")[0]
    c, t = int(r["Calls"]), float(r["TotalDurationNs"])
    a = rows.setdefault(k, [0, 0.0])
    a[0] += c
    a[1] += t
frames = rows.get("k_wave_init", [1, 0])[0]
parts = []
total = 0.0
for k in ("k_trace2", "k_shade2", "k_shade2m", "k_res2d", "k_res2md", "k_wave_init", "k_accumulate"):
    if k in rows:
        c, t = rows[k]
        parts.append(f"{k} {t / c / 1e3:.1f}us x{c / frames:.0f}")
for k, (c, t) in rows.items():
    if k.startswith("k_"):
        total += t
print(f"{v:50s} frame {total / frames / 1e6:.3f} ms  " + "  ".join(parts))
