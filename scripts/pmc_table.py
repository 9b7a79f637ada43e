#!/usr/bin/env python3
"""Per-kernel mean (over dispatches) of every counter in gpurun_out/pmc_<tag>/run_counter_collection.csv.
usage: scripts/pmc_table.py <tag> [<tag> ...]"""
import collections
import csv
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def table(tag):
    f = os.path.join(ROOT, "gpurun_out", f"pmc_{tag}", "run_counter_collection.csv")
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    return {k: {c: v / len(disp[k]) for c, v in d.items()} for k, d in per.items()}


if __name__ == "__main__":
    merged = collections.defaultdict(dict)
    for tag in sys.argv[1:]:
        for k, d in table(tag).items():
            merged[k].update(d)
    for k, d in merged.items():
        if k.startswith("prt::"):
            print(k)
            for c, v in sorted(d.items()):
                print(f"   {c:28s} {v:16.4g}")
