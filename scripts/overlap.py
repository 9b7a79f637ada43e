#!/usr/bin/env python3
"""Concurrency in a rocprofv3 --kernel-trace session (diagnostic for frames in flight): per hardware queue the
dispatches and their kernels; the time with >= 2 kernels running; for k_trace2, the share of its dispatch time that
overlapped another kernel.  usage: scripts/overlap.py <kernel_trace.csv> [--last-ms T] (only the last T ms)"""
import collections
import csv
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").split("::")[-1].split("<")[0]
    q = r.get("Queue_Id") or r.get("Queue_ID") or "?"
    s = r.get("Stream_Id") or r.get("Stream_ID") or "?"
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, q, s))
rows.sort()
if "--last-ms" in sys.argv:
    t = float(sys.argv[sys.argv.index("--last-ms") + 1]) * 1e6
    end = max(e for _, e, *_ in rows)
    rows = [r for r in rows if r[0] >= end - t]
per_q = collections.defaultdict(collections.Counter)
for s_, e, n, q, st in rows:
    per_q[(q, st)][n] += 1
for k, c in sorted(per_q.items()):
    print("queue", k[0], "stream", k[1], dict(c.most_common(6)))
ev = []
for s_, e, n, *_ in rows:
    ev.append((s_, 1))
    ev.append((e, -1))
ev.sort()
active, last, multi = 0, ev[0][0], 0
for t, d in ev:
    if active >= 2:
        multi += t - last
    active += d
    last = t
span = ev[-1][0] - ev[0][0]
print(f"span {span / 1e6:.3f} ms, >= 2 kernels running {multi / 1e6:.3f} ms ({multi / span:.2f})")
tr = [(s_, e) for s_, e, n, *_ in rows if n == "k_trace2"]
others = [(s_, e) for s_, e, n, *_ in rows]
ov = tot = 0
for a, b in tr:
    tot += b - a
    cov = 0
    for c, d in others:
        if (c, d) == (a, b):
            continue
        lo, hi = max(a, c), min(b, d)
        if hi > lo:
            cov = max(cov, hi - lo)
    ov += cov
print(f"k_trace2: {len(tr)} dispatches, {tot / 1e6:.3f} ms, the longest overlap per dispatch sums to {ov / 1e6:.3f} ms")
