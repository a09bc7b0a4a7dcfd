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
    if "MRP_SCHEDULE" in os.environ:   # 0 lane order, 1 costliest-first dispatch (lane blocks then mix)
        b.set_schedule(int(os.environ["MRP_SCHEDULE"]))
    b.reset()
    for _ in range(warmup):
        b.step()
    L = _native.load()
    tr = np.zeros((lanes, _native.trace_words()), np.uint32)
    acc = np.zeros((lanes, _native.trace_words()), np.float64)
    slow_block = np.zeros((lanes + 1023) // 1024, np.int64)
    last_block = np.zeros_like(slow_block)
    launches = []
    for _ in range(steps):
        b.step()
        assert L.mrp_debug_trace(0, tr.ctypes.data_as(ctypes.c_void_p), lanes) == 0
        acc += tr
        slow_block[int(np.argmax(tr[:, 11])) // 1024] += 1
        # words 28/29: s_memrealtime (100 MHz) at the lane's entry and end, low 32 bits
        t0 = tr[:, 28].astype(np.int64)
        ref = int(t0.min())
        start = ((t0 - ref) & 0xffffffff) * 0.01          # us after the launch's first lane started
        end = ((tr[:, 29].astype(np.int64) - ref) & 0xffffffff) * 0.01
        last = int(np.argmax(end))
        hw, xcc = tr[:, 30].astype(np.int64), tr[:, 31].astype(np.int64) & 0xf
        simd_key = (xcc << 16) | (((hw >> 13) & 7) << 12) | (((hw >> 12) & 1) << 11) | (((hw >> 8) & 0xf) << 4) | ((hw >> 4) & 3)
        share = np.nonzero(simd_key == simd_key[last])[0]
        last_block[last // 1024] += 1
        launches.append({"span_us": float(end.max()), "last_lane": last, "last_block": last // 1024,
                         "last_start_us": float(start[last]), "last_duration_us": float(end[last] - start[last]),
                         "last_cycles": int(tr[last, 11]), "slowest_duration_lane": int(np.argmax(tr[:, 11])),
                         "slowest_duration_us": float((end - start).max()),
                         "simd_mates": [{"lane": int(m), "start_us": float(start[m]), "end_us": float(end[m])} for m in share if m != last],
                         "late_start_us_mean": float(start[3072:].mean()) if lanes > 3072 else None})
    acc /= steps
    res = {"env": env, "lanes": lanes, "launches": launches, "blocks": []}
    sp = np.array([l["span_us"] for l in launches])
    print(f"launch span (first lane start to last lane end) {sp.mean():.1f} us mean; the last lane to end was in block "
          + " ".join(f"{k}:{int(v)}" for k, v in enumerate(last_block)) + f"; its start {np.mean([l['last_start_us'] for l in launches]):.1f} us, "
          f"duration {np.mean([l['last_duration_us'] for l in launches]):.1f} us; longest lane duration {np.mean([l['slowest_duration_us'] for l in launches]):.1f} us")
    for l in launches[:3]:
        print(f"  launch: span {l['span_us']:.1f} last lane {l['last_lane']} start {l['last_start_us']:.1f} dur {l['last_duration_us']:.1f}; SIMD mates "
              + ", ".join(f"{m['lane']}:{m['start_us']:.0f}-{m['end_us']:.0f}" for m in l["simd_mates"]))
    for k in range(len(slow_block)):
        blk = acc[k * 1024:(k + 1) * 1024]
        res["blocks"].append({"lanes": [k * 1024, min(lanes, (k + 1) * 1024) - 1], "slowest_lane_launches": int(slow_block[k]),
                              "mean_total": float(blk[:, 11].mean()),
                              "mean_phases": {n: float(blk[:, i].mean()) for i, n in enumerate(NAMES)},
                              # load sub-phases, cycles from the wave's start: state loaded, tables loaded, barrier
                              "load_marks": [float(blk[:, 24].mean()), float(blk[:, 25].mean()), float(blk[:, 26].mean())],
                              # collide split: narrow phase, serial commit (cycles)
                              "collide_split": [float(blk[:, 22].mean()), float(blk[:, 23].mean())],
                              # TOI split: candidate scan + b2TimeOfImpact, events (cycles)
                              "toi_split": [float(blk[:, 20].mean()), float(blk[:, 21].mean())],
                              "last_to_end_launches": int(last_block[k])})
        p = res["blocks"][-1]["mean_phases"]
        print(f"lanes {k * 1024:5d}-{min(lanes, (k + 1) * 1024) - 1:5d}: slowest in {slow_block[k]:2d}/{steps} launches, "
              f"last to end in {last_block[k]:2d}, "
              f"mean total {blk[:, 11].mean():9.0f}  load {p['load+act']:8.0f}  solve {p['solve(islands)']:8.0f}  "
              f"TOI {p['TOI']:8.0f}  store {p['store']:8.0f} (collide: narrow {blk[:, 22].mean():7.0f} commit {blk[:, 23].mean():7.0f})  load marks "
              + " ".join(f"{v:8.0f}" for v in res["blocks"][-1]["load_marks"])
              + f"  TOI split {blk[:, 20].mean():7.0f} / {blk[:, 21].mean():7.0f}")
    if out:
        with open(out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
