"""Per-lane phase cycles by lane (workgroup) index over bench.py's window (diagnostic; stamps build).

    MRP_LIB=gym_puzzles_amd/libmrp_stamps.so python tools/lane_phases.py ENV LANES [WARMUP STEPS OUT.json]

Workgroup b steps lane b, and at 3 waves per SIMD only the first 3072 workgroups are resident at
once, so lanes are grouped in blocks of 1024 by index: the phase means of each block (all
lane-steps) and how often a block holds the launch's slowest lane.
"""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from gym_puzzles_amd import Batch, _native  # noqa: E402

NAMES = ["load+act", "apply_actions", "FNC(new fixtures)", "collide", "solve(islands)", "FNC(after solve)",
         "TOI", "obs/reward", "outputs", "auto-reset", "store"]


def main():
    env, lanes = int(sys.argv[1]), int(sys.argv[2])
    warmup = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    out = sys.argv[5] if len(sys.argv) > 5 else None
    b = Batch(env, lanes, seed=17)
    b.set_auto_reset(True)
    b.reset()
    for _ in range(warmup):
        b.step()
    L = _native.load()
    tr = np.zeros((lanes, 32), np.uint32)
    acc = np.zeros((lanes, 32), np.float64)
    slow_block = np.zeros((lanes + 1023) // 1024, np.int64)
    for _ in range(steps):
        b.step()
        assert L.mrp_debug_trace(0, tr.ctypes.data_as(ctypes.c_void_p), lanes) == 0
        acc += tr
        slow_block[int(np.argmax(tr[:, 11])) // 1024] += 1
    acc /= steps
    res = {"env": env, "lanes": lanes, "blocks": []}
    for k in range(len(slow_block)):
        blk = acc[k * 1024:(k + 1) * 1024]
        res["blocks"].append({"lanes": [k * 1024, min(lanes, (k + 1) * 1024) - 1], "slowest_lane_launches": int(slow_block[k]),
                              "mean_total": float(blk[:, 11].mean()),
                              "mean_phases": {n: float(blk[:, i].mean()) for i, n in enumerate(NAMES)},
                              # load sub-phases, cycles from the wave's start: state loaded, tables loaded, barrier
                              "load_marks": [float(blk[:, 24].mean()), float(blk[:, 25].mean()), float(blk[:, 26].mean())]})
        p = res["blocks"][-1]["mean_phases"]
        print(f"lanes {k * 1024:5d}-{min(lanes, (k + 1) * 1024) - 1:5d}: slowest in {slow_block[k]:2d}/{steps} launches, "
              f"mean total {blk[:, 11].mean():9.0f}  load {p['load+act']:8.0f}  solve {p['solve(islands)']:8.0f}  "
              f"TOI {p['TOI']:8.0f}  store {p['store']:8.0f}  load marks " + " ".join(f"{v:8.0f}" for v in res["blocks"][-1]["load_marks"]))
    if out:
        with open(out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
