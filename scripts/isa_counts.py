#!/usr/bin/env python3
"""Per-visit ISA instruction counts of the traversal's two inner operations (scripts/isa_counts.hip) on gfx950,
compiled with the product's device flags: writes profiles/isa_counts.json.  The kernels wrap exactly one
node8_hits / mt_test; their prologue (argument and ray loads) is reported separately from the body."""
import collections
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FLAGS = ["-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-fno-slp-vectorize", "--offload-arch=gfx950",
         "-fno-gpu-rdc", "--cuda-device-only", "-S"]


def main():
    out = "/tmp/isa_counts.s"
    subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, os.path.join(ROOT, "scripts", "isa_counts.hip"), "-o", out],
                   check=True)
    text = open(out).read().splitlines()
    res = {"flags": " ".join(FLAGS[:-2]), "kernels": {}}
    for name, label in (("k_isa_node8", "node8_hits (one Node8 visit: 8 child slabs)"),
                        ("k_isa_tri", "mt_test (one Moeller-Trumbore leaf test)")):
        start = next(i for i, l in enumerate(text) if re.match(rf"^_Z\w*{name}\w*:", l))
        end = next(i for i in range(start, len(text)) if "s_endpgm" in text[i])
        ins = [l.split()[0] for l in text[start + 1:end] if re.match(r"^\s+[a-z]", l) and not l.strip().startswith(";")]
        c = collections.Counter(ins)
        valu = {k: v for k, v in c.items() if k.startswith("v_")}
        res["kernels"][name] = {
            "what": label,
            "valu": sum(valu.values()),
            "salu": sum(v for k, v in c.items() if k.startswith("s_") and not k.startswith("s_waitcnt")),
            "vmem_loads": sum(v for k, v in c.items() if k.startswith("global_load") or k.startswith("buffer_load")),
            "smem_loads": sum(v for k, v in c.items() if k.startswith("s_load")),
            "by_op": dict(sorted(valu.items(), key=lambda kv: -kv[1])),
        }
    path = os.path.join(ROOT, "profiles", "isa_counts.json")
    with open(path, "w") as f:
        json.dump(res, f, indent=1)
    for k, d in res["kernels"].items():
        print(k, "VALU", d["valu"], "SALU", d["salu"], "loads", d["vmem_loads"])


if __name__ == "__main__":
    sys.exit(main())
