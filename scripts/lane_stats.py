#!/usr/bin/env python3
"""Lane-usage histogram of the persistent traversal: run with the PRT_LANE_STATS diagnostic build
(prt/ab/libprt_lanestats.so copied over prt/libprt.so by scripts/gpu_lanestats.sh).  Renders the C4 frame at
world 1 and rank 0's world-8 share with stats, parses the per-launch counter rows the library prints
("prt: lanestats <launch> c0..c31", prt_persist.h) and writes profiles/<tag>_lane_stats.json.

Counters per launch (summed over waves): 0 main-loop iterations, 1 active lanes, 2 lanes in node_step, 3 lanes
in tri_step, 4 iterations running node_step, 5 iterations running tri_step, 6 iterations running both,
7 iterations with a lane between BLASes / finishing, 8-16 histogram of node lanes per iteration (bucket
ceil(n/8)), 17-25 the same for tri lanes, 26 tail iterations, 27/28 tail node / tri lanes, 29/30 tail iterations
running node / tri, 31 waves."""
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VALU_NODE, VALU_TRI = 190, 67  # static VALU of one node visit / triangle test (profiles/isa_counts.json)


def child(world, path):
    code = f"""
import sys, numpy as np, torch
sys.path.insert(0, {os.path.join(ROOT, 'physically-based-ray-tracer_amd')!r})
import prt
from prt import scenes
sd = scenes.config_c4(); W, H = 1920, 1080
c = prt.Context(0)
c.set_scene(prt.Scene.from_data(sd)); c.set_camera(prt.Camera(sd.cam_pos, sd.cam_target, np.float32(W) / np.float32(H)))
if {world} == 1:
    c.render(W, H, 4, 4, stats=True)
    print('MEASURE', file=sys.stderr, flush=True)
    c.render(W, H, 4, 4, stats=True)
else:
    per = c.tile_buffer_pixels(W, H, 32, {world})
    t = torch.zeros((per, 4), dtype=torch.float32, device='cuda')
    c.render_tiles(W, H, 4, 4, 32, 0, {world}, t.data_ptr(), stats=True)
    print('MEASURE', file=sys.stderr, flush=True)
    c.render_tiles(W, H, 4, 4, 32, 0, {world}, t.data_ptr(), stats=True)
c.close()
"""
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    if r.returncode != 0:
        sys.stderr.write(r.stderr[-3000:])
        raise SystemExit(r.returncode)
    err = r.stderr.split("MEASURE", 1)[1]
    with open(path, "w") as f:
        f.write(err)
    rows = {}
    for m in re.finditer(r"prt: lanestats (\d+)((?: \d+){32})", err):
        rows[int(m.group(1))] = [int(x) for x in m.group(2).split()]
    return rows


def summarize(rows):
    out = []
    tot = [0] * 32
    for i in sorted(rows):
        r = rows[i]
        tot = [a + b for a, b in zip(tot, r)]
        out.append(derive(r, i))
    return out, derive(tot, "all")


def derive(r, launch):
    it, act, nn, nt, itn, itt, itb, itd = r[:8]
    tit, tnn, tnt, titn, titt = r[26:31]
    issued = itn * VALU_NODE + itt * VALU_TRI          # wave-instructions the two branches issue (main loop)
    useful = (nn * VALU_NODE + nt * VALU_TRI) / 64.0    # lane-instructions / 64
    tissued = titn * VALU_NODE + titt * VALU_TRI
    tuseful = (tnn * VALU_NODE + tnt * VALU_TRI) / 64.0
    return {
        "launch": launch, "waves": r[31], "iterations": it, "tail_iterations": tit,
        "mean_active_lanes": act / max(it, 1), "mean_node_lanes": nn / max(it, 1), "mean_tri_lanes": nt / max(it, 1),
        "frac_iters_node": itn / max(it, 1), "frac_iters_tri": itt / max(it, 1), "frac_iters_both": itb / max(it, 1),
        "frac_iters_blas_end": itd / max(it, 1),
        "node_lanes_hist_by8": r[8:17], "tri_lanes_hist_by8": r[17:26],
        "branch_lane_efficiency_main": useful / max(issued, 1),
        "branch_lane_efficiency_tail": tuseful / max(tissued, 1),
        "tail_share_of_branch_issue": tissued / max(issued + tissued, 1),
        "mean_tail_node_lanes": tnn / max(tit, 1), "mean_tail_tri_lanes": tnt / max(tit, 1),
    }


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r04"
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    res = {"valu_node": VALU_NODE, "valu_tri": VALU_TRI}
    for world in (1, 8):
        rows = child(world, os.path.join(ROOT, "gpurun_out", f"lanestats_w{world}.log"))
        per, tot = summarize(rows)
        res[f"world{world}"] = {"total": tot, "per_launch": per}
        print(f"world {world}: " + json.dumps(tot), flush=True)
    with open(os.path.join(ROOT, "profiles", f"{tag}_lane_stats.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
