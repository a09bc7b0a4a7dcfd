"""Issue-count roofline of k_step from the replayed slowest lane-steps (CPU; reads gpurun_out/).

    python tools/issue_roofline.py DIR OUT.json [ENV ...]

For each config, DIR holds (tools/sessions/r4_session2.sh): cap_env<E>.npz (the 20 slowest lane-steps of the
driver window with their in-batch phase traces), replay_stamps_env<E>.json (the same lane-steps
stepped alone by the stamps library), pmc_env<E>/ (rocprofv3 SQ_INSTS_* counters of each lone
replay: exactly that lane-step's executed instructions) and kt_env<E>/ (their lone-wave durations).

A lone wave issues one instruction per 4 cycles whatever its type (MI355X_MICROARCH.md, row
'vector-instruction ISSUE cost'; s_nop 0 costs the same 4, SQ_INSTS counts it as SALU), so

    issue floor of a lane-step = 4 x SQ_INSTS cycles

and the launch, whose duration is its slowest lane's, cannot end before its slowest lane's issue
floor at the clock the chip holds.  Per config this writes: the mean over the 20 launches of the
slowest lane's instruction mix and issue floor (cycles and us at the in-kernel clock), the same
lane-step's lone-wave duration (kernel trace; stamps total) and its in-batch duration (stamps
trace), and the phase split alone vs in the batch.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict

import numpy as np

PHASES = ["load+act", "apply_actions", "FNC(new fixtures)", "collide", "solve(islands)", "FNC(after solve)",
          "TOI", "obs/reward", "outputs", "auto-reset", "store"]
SUB = {"velocity_sweeps": 16, "position_passes": 17, "island_setup": 18}
COUNTERS = ("SQ_INSTS", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH",
            "SQ_INSTS_VMEM", "SQ_WAVE_CYCLES")


def kstep_pmc(d):
    per = defaultdict(dict)
    names = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_step" not in r["Kernel_Name"]:
                continue
            i = int(r["Dispatch_Id"])
            per[i][r["Counter_Name"]] = float(r["Counter_Value"])
            names[i] = r["Kernel_Name"]
    return [per[i] for i in sorted(per)]


def kstep_durations(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_step" in r["Kernel_Name"]:
                rows.append((int(r["Dispatch_Id"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3))
    return [us for _, us in sorted(rows)]


def one(d, env):
    cap = np.load(os.path.join(d, f"cap_env{env}.npz"))
    n = len(cap["lane"])
    tb = cap["trace"].astype(np.float64)                      # in-batch traces of the slowest lanes
    rep = json.load(open(os.path.join(d, f"replay_stamps_env{env}.json")))["rows"]
    ta = np.array([r["trace_alone"] for r in rep], np.float64)
    pmc = kstep_pmc(os.path.join(d, f"pmc_env{env}"))
    dur = kstep_durations(os.path.join(d, f"kt_env{env}"))
    assert len(pmc) == n, (len(pmc), n)
    reps = len(dur) // n
    dur = np.array(dur[:n * reps]).reshape(n, reps).min(axis=1)   # lone-wave duration, best of the repeats
    cand = [os.path.join(d, f"r4_phase_env{env}.json"), os.path.join(d, "..", f"r4_phase_env{env}.json")]
    ph = next((json.load(open(c)) for c in cand if os.path.exists(c)), None)
    ghz = ph["s_memtime_ghz"] if ph else 2.2
    inst = {c: np.array([p.get(c, np.nan) for p in pmc]) for c in COUNTERS}
    floor_cyc = 4.0 * inst["SQ_INSTS"]
    res = {
        "env": env, "lanes": int(cap["lanes"]), "timed_steps_after_spawn": [int(cap["warmup"]) + 1, int(cap["warmup"] + cap["steps"])],
        "launches": n, "in_kernel_clock_ghz": ghz,
        "slowest_lane_instructions_mean": {c: float(np.nanmean(v)) for c, v in inst.items() if c != "SQ_WAVE_CYCLES"},
        "issue_floor_cycles_mean": float(floor_cyc.mean()),
        "issue_floor_us_mean": float(floor_cyc.mean() / ghz / 1e3),
        "lone_wave_duration_us_mean": float(dur.mean()),
        "lone_wave_stamps_cycles_mean": float(ta[:, 11].mean()),
        "in_batch_stamps_cycles_mean": float(tb[:, 11].mean()),
        "issue_floor_over_lone_wave": float(floor_cyc.mean() / ta[:, 11].mean()),
        "issue_floor_over_in_batch": float(floor_cyc.mean() / tb[:, 11].mean()),
        "phases_alone_cycles_mean": {p: float(ta[:, i].mean()) for i, p in enumerate(PHASES)},
        "phases_in_batch_cycles_mean": {p: float(tb[:, i].mean()) for i, p in enumerate(PHASES)},
        "solve_split_alone_cycles_mean": {k: float(ta[:, w].mean()) for k, w in SUB.items()},
        "solve_split_in_batch_cycles_mean": {k: float(tb[:, w].mean()) for k, w in SUB.items()},
        "slowest_lane_work_mean": {"island_contacts": float(tb[:, 12].mean()), "toi_events": float(tb[:, 13].mean()),
                                   "position_passes": float(tb[:, 14].mean()), "velocity_updates": float(tb[:, 15].mean())},
    }
    return res


def main():
    d, out = sys.argv[1], sys.argv[2]
    envs = [int(e) for e in sys.argv[3:]] or [0, 1, 2, 4, 5]
    res = {}
    for e in envs:
        r = one(d, e)
        # keyed like bench.py's run: env, lanes, first and last timed step after spawn, seed
        res[f"{e}:{r['lanes']}:{r['timed_steps_after_spawn'][0]}:{r['timed_steps_after_spawn'][1]}:17"] = r
        i = r["slowest_lane_instructions_mean"]
        print(f"env {e}: slowest lane-step {i['SQ_INSTS']:.0f} instr (VALU {i['SQ_INSTS_VALU']:.0f} SALU {i['SQ_INSTS_SALU']:.0f} "
              f"LDS {i['SQ_INSTS_LDS']:.0f} SMEM {i['SQ_INSTS_SMEM']:.0f} BR {i['SQ_INSTS_BRANCH']:.0f} VMEM {i['SQ_INSTS_VMEM']:.0f}); "
              f"issue floor {r['issue_floor_cycles_mean']:.0f} cyc = {r['issue_floor_us_mean']:.1f} us; alone {r['lone_wave_stamps_cycles_mean']:.0f} cyc "
              f"({r['lone_wave_duration_us_mean']:.1f} us trace), in batch {r['in_batch_stamps_cycles_mean']:.0f} cyc; "
              f"floor/alone {r['issue_floor_over_lone_wave']:.2f} floor/batch {r['issue_floor_over_in_batch']:.2f}")
        for p in PHASES:
            a, b = r["phases_alone_cycles_mean"][p], r["phases_in_batch_cycles_mean"][p]
            if max(a, b) > 0.01 * r["in_batch_stamps_cycles_mean"]:
                print(f"    {p:18s} alone {a:9.0f}  batch {b:9.0f}")
        for k in SUB:
            print(f"    solve/{k:16s} alone {r['solve_split_alone_cycles_mean'][k]:9.0f}  batch {r['solve_split_in_batch_cycles_mean'][k]:9.0f}")
    with open(out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
