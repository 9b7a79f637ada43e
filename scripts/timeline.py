#!/usr/bin/env python3
"""Render-stream timeline of a rocprofv3 --kernel-trace session (its kernel_trace.csv): per kernel name, the
dispatches, total and mean duration; the idle time of the GPU (no kernel of any queue running); and, for one
kernel (--focus, default k_build_small), how much of each of its dispatches ran while no other kernel ran.
usage: scripts/timeline.py <kernel_trace.csv> [--focus NAME]"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    focus = sys.argv[sys.argv.index("--focus") + 1] if "--focus" in sys.argv else "k_build_small"
    rows = []
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if "(anonymous namespace)::" in name:
            name = name.split("(anonymous namespace)::")[1]
        name = name.split("(")[0].replace("void ", "").split("::")[-1].split("<")[0]
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    if "--window" in sys.argv:  # only the dispatches inside [start, end] ms after the first
        a, b = (float(x) for x in sys.argv[sys.argv.index("--window") + 1].split(":"))
        base = rows[0][0]
        rows = [r for r in rows if a * 1e6 <= r[0] - base <= b * 1e6]
    t0, t1 = rows[0][0], max(e for _, e, _ in rows)
    per = collections.defaultdict(list)
    for s, e, n in rows:
        per[n].append(e - s)
    # union of busy intervals
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in rows:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    print(f"span {(t1 - t0) / 1e6:.3f} ms, GPU busy {busy / 1e6:.3f} ms, idle {(t1 - t0 - busy) / 1e6:.3f} ms")
    # concurrency: time with k kernels running at once
    edges = sorted([(s, 1) for s, _, _ in rows] + [(e, -1) for _, e, _ in rows])
    conc = collections.Counter()
    k, last = 0, edges[0][0]
    for t, d in edges:
        conc[k] += t - last
        k += d
        last = t
    print("  time with k kernels running: " + ", ".join(f"{k}: {v / 1e6:.3f} ms" for k, v in sorted(conc.items())))
    for n, d in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {n:28s} {len(d):6d} dispatches  total {sum(d) / 1e6:9.3f} ms  mean {sum(d) / len(d) / 1e3:9.1f} us")
    alone = []
    for s, e, n in rows:
        if n != focus:
            continue
        # time of [s, e) not covered by any other kernel
        cov = sorted((max(s, s2), min(e, e2)) for s2, e2, n2 in rows if n2 != focus and s2 < e and e2 > s)
        c, ce = 0, s
        for a, b in cov:
            if b <= ce:
                continue
            c += b - max(a, ce)
            ce = b
        alone.append((e - s - c) / 1e3)
    if alone:
        alone.sort()
        print(f"{focus}: {len(alone)} dispatches, alone on the GPU median {alone[len(alone) // 2]:.1f} us, "
              f"max {alone[-1]:.1f} us, total {sum(alone) / 1e3:.3f} ms")
    # traversal launches far above their median (--slow FACTOR, default 1.6): how many, and what overlapped them
    fac = float(sys.argv[sys.argv.index("--slow") + 1]) if "--slow" in sys.argv else 1.6
    tr = [(s, e) for s, e, n in rows if n == "k_trace2"]
    if tr:
        med = sorted(e - s for s, e in tr)[len(tr) // 2]
        slow = [(s, e) for s, e in tr if e - s > fac * med]
        lone = sum(1 for s, e in slow if not any(n2 != "k_trace2" and s2 < e and e2 > s for s2, e2, n2 in rows))
        print(f"k_trace2: {len(tr)} launches, median {med / 1e3:.1f} us; {len(slow)} above {fac} x the median "
              f"({lone} with no other kernel overlapping)")


if __name__ == "__main__":
    main()
