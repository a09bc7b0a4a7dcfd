"""VALU and latency rooflines of k_step from the oracle's op counts (CPU only).

The oracle (oracle/b2_oracle.c, work model OrWork) counts, for every lane and launch of the exact
bench.py workload (seed, lanes, step window), the solver work the device runs: velocity contact
updates by point count (sweeps counted with the device's exact early exit), position point
updates, narrow-phase polygon pairs, b2TimeOfImpact calls and TOI islands.  Each unit is priced
with the float operations of its code (counted below from the oracle's source, which performs the
device's operations in the same order) and with the length of its dependent chain:

* flops per launch (all lanes)             -> roofline.valu    = flops / kernel time / 157.3 TF
* dependent ops of the slowest lane's chain -> roofline.latency = ops x 6 cycles (one wave's
  dependent f32 VALU latency, tools/micro/latbench.hip) / 2.4 GHz / kernel time

Writes profiles/<tag>_valu_latency.json; bench.py reads the entry whose key matches its run
(env, lanes, first and last timed step after spawn, seed) and divides by its live kernel_ms.

    python tools/roofline_model.py <tag> [env:lanes:first:last ...]
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)

from gym_puzzles_amd.spawn import draw_bounds  # noqa: E402
from oracle.oracle import WORK_NAMES, batch_work  # noqa: E402

W = {n: i for i, n in enumerate(WORK_NAMES)}

# float operations per unit (f32 add/sub/mul/div, plus the f64 ops of b2Rot::Set; compares and
# selects not counted), from oracle/b2_oracle.c:
#   velocity update (solver_solve_velocity): friction row 37 per point; normal row 37 (1 point) or
#     the 2-point block solve 78 (dv 20, vn 6, b 10, x 6, d 2, impulses 4, bodies 30)
#   position point (solver_solve_position + psm_init): 85 f32 + one b2Rot::Set (24 f64 flops: 14
#     ops, 10 of them FMAs) for the body whose angle moved
#   narrow phase (collide_polygons, 8-gon x 4-gon): two b2FindMaxSeparation (~490), clipping and
#     the manifold (~110)
#   b2TimeOfImpact: GJK iterations, separation functions and the root finder, ~1500 per call
#   TOI island set-up and solver init: 120 per contact point (b2WorldManifold, masses)
FLOPS = {"vel_upd1": 74, "vel_upd2": 152, "toi_vel_upd": 152, "pos_points": 109, "toi_pos_points": 109,
         "sat_calls": 600, "toi_calls": 1500}
# dependent ops on a lane's critical path per unit (the operations each update waits on in
# sequence: friction row 16 per point, 1-point normal row 14, 2-point block solve 20; position point
# 40 f32 + the 14-op f64 b2Rot::Set chain)
DEP = {"vel_upd1": 30, "vel_upd2": 52, "toi_vel_upd": 52, "pos_points": 54, "toi_pos_points": 54}
DEP_CYCLES = 6.0          # one wave's dependent f32 VALU latency (tools/micro/latbench.hip)
CLOCK_HZ = 2.4e9          # MI355X_MICROARCH.md max clock
VALU_PEAK = 157.3e12      # FP32 vector, MI355X_MICROARCH.md chip table


def model(env: int, lanes: int, first: int, last: int, seed: int = 17) -> dict:
    w = batch_work(env, lanes, last, seed, draw_bounds(env), threads=os.cpu_count() or 1)[first - 1:last]
    n = w.shape[0]
    flops = sum(FLOPS[k] * w[..., W[k]].sum() for k in FLOPS) / n
    dep = sum(DEP[k] * w[..., W[k]] for k in DEP)            # [steps, lanes]
    slow = dep.max(axis=1)
    tot = w.sum(axis=(0, 1))
    return {"env": env, "lanes": lanes, "steps_after_spawn": [first, last], "seed": seed,
            "flops_per_launch": float(flops),
            "slowest_lane_dependent_ops_per_launch": float(slow.mean()),
            "latency_floor_ms": float(slow.mean() * DEP_CYCLES / CLOCK_HZ * 1e3),
            "work_per_launch": {k: float(tot[W[k]] / n) for k in FLOPS},
            "constants": {"flops": FLOPS, "dependent_ops": DEP, "dependent_cycles": DEP_CYCLES, "clock_hz": CLOCK_HZ,
                          "valu_peak_flops": VALU_PEAK}}


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r3"
    keys = sys.argv[2:] or ["0:4096:6:25", "0:4096:21:220", "1:4096:6:25", "2:1024:6:25", "4:1024:6:25", "5:4096:6:25"]
    out = {}
    for k in keys:
        e, lanes, a, b = (int(x) for x in k.split(":"))
        m = model(e, lanes, a, b)
        out[f"{e}:{lanes}:{a}:{b}:17"] = m
        print(k, json.dumps({x: m[x] for x in ("flops_per_launch", "slowest_lane_dependent_ops_per_launch",
                                              "latency_floor_ms")}), flush=True)
    path = os.path.join(ROOT, "profiles", f"{tag}_valu_latency.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("wrote", path)


if __name__ == "__main__":
    main()
