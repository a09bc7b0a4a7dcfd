"""Per-phase time split of k_step (diagnostic build with -DMRP_STAMPS), over bench.py's window.

    python -m gym_puzzles_amd.build --variant gym_puzzles_amd/libmrp_stamps.so 0 1 2 4 5 -DMRP_STAMPS
    MRP_LIB=gym_puzzles_amd/libmrp_stamps.so python tools/phase_profile.py ENV LANES [WARMUP STEPS OUT.json]

Thread 0 of each lane stamps s_memtime at phase boundaries (mrp_world.h MRP_STAMP / MRP_SUB).  The
launch's duration is its slowest lane's, so besides the mean over all lane-steps this records, for
every timed launch, the phases of that launch's slowest lane (read back with mrp_debug_trace after
each launch) and averages them over the window: the table that says where a launch's time goes.
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
# trace words: 0-10 phases, 11 total, 12 island contacts, 13 TOI events, 14 position passes, 15 velocity
# updates run, 16 velocity-sweep cycles, 17 position-pass cycles, 18 island set-up cycles (thread 0),
# 19 largest island's contact count, 20/21 TOI split (scan + b2TimeOfImpact, events), 22/23 collide split (narrow phase, commit)
SUB = {"velocity_sweeps": 16, "position_passes": 17, "island_setup": 18}
# round 6 (trace rows of 40 words): the solve's thread-0 bookkeeping and the TOI scan alone
SUB2 = {"island_building": 32, "island_writeback_integrate": 33, "fixture_sync": 34}
TOI_SCAN = 35


def main():
    env = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    lanes = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    warmup = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    out = sys.argv[5] if len(sys.argv) > 5 else None
    b = Batch(env, lanes, seed=17)
    b.set_auto_reset(True)
    b.reset()
    for _ in range(warmup):
        b.step()
    L = _native.load()
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    buf = np.zeros(16, np.uint64)
    pmax, smax, rt = np.zeros(16, np.uint64), np.zeros(256, np.uint64), np.zeros(2, np.uint64)
    assert L.mrp_debug_stamps(0, vp(buf)) == 0, "not a -DMRP_STAMPS build of this env"
    L.mrp_debug_stamps_ext(0, vp(pmax), vp(smax), vp(rt))
    tr = np.zeros((lanes, _native.trace_words()), np.uint32)
    slow = []          # per launch: the slowest lane's trace row
    slow10 = []        # per launch: mean trace row of the 10 slowest lanes
    for _ in range(steps):
        b.step()
        L.mrp_debug_trace(0, vp(tr), lanes)
        order = np.argsort(-tr[:, 11].astype(np.int64))
        slow.append(tr[order[0]].astype(np.int64))
        slow10.append(tr[order[:10]].astype(np.float64).mean(axis=0))
    L.mrp_debug_stamps(0, vp(buf))
    L.mrp_debug_stamps_ext(0, vp(pmax), vp(smax), vp(rt))
    ghz = 0.1 * rt[0] / max(rt[1], 1)   # s_memrealtime ticks at 100 MHz
    slow = np.array(slow)
    slow10 = np.array(slow10)
    tot_mean = buf[:11].astype(np.float64).sum() / lanes / steps
    res = {"env": env, "lanes": lanes, "timed_steps_after_spawn": [warmup + 1, warmup + steps],
           "s_memtime_ghz": float(ghz),
           "mean_lane_step_cycles": float(tot_mean),
           "mean_lane_step_phases": {n: float(buf[i]) / lanes / steps for i, n in enumerate(NAMES)},
           "slowest_lane_per_launch": {
               "total_cycles_mean": float(slow[:, 11].mean()), "total_cycles_max": int(slow[:, 11].max()),
               "total_us_mean": float(slow[:, 11].mean() / ghz / 1e3),
               "phases_cycles_mean": {n: float(slow[:, i].mean()) for i, n in enumerate(NAMES)},
               "solve_split_cycles_mean": {k: float(slow[:, w].mean()) for k, w in SUB.items()},
               "solve_bookkeeping_cycles_mean": ({k: float(slow[:, w].mean()) for k, w in SUB2.items()}
                                                 if slow.shape[1] > 35 else None),
               "toi_scan_alone_cycles_mean": float(slow[:, TOI_SCAN].mean()) if slow.shape[1] > 35 else None,
               "island_contacts_mean": float(slow[:, 12].mean()), "toi_events_mean": float(slow[:, 13].mean()),
               "position_passes_mean": float(slow[:, 14].mean()), "velocity_updates_mean": float(slow[:, 15].mean()),
               "largest_island_contacts_mean": float(slow[:, 19].mean()),
               # TOI phase split: candidate scan + b2TimeOfImpact of every candidate, then the events
               # (TOI island, sub-step solve, FindNewContacts)
               "toi_split_cycles_mean": {"scan_and_time_of_impact": float(slow[:, 20].mean()), "events": float(slow[:, 21].mean())},
               # collide split: contact-list snapshot + narrow phase of every contact, then thread 0's commit
               "collide_split_cycles_mean": {"narrow_phase": float(slow[:, 22].mean()), "serial_commit": float(slow[:, 23].mean())}},
           "ten_slowest_lanes_per_launch": {
               "total_cycles_mean": float(slow10[:, 11].mean()),
               "phases_cycles_mean": {n: float(slow10[:, i].mean()) for i, n in enumerate(NAMES)},
               "solve_split_cycles_mean": {k: float(slow10[:, w].mean()) for k, w in SUB.items()}}}
    s = res["slowest_lane_per_launch"]
    print(f"env {env} lanes {lanes} steps {warmup + 1}-{warmup + steps}: clock {ghz:.3f} GHz, mean lane-step "
          f"{tot_mean:.0f} cyc, slowest lane per launch {s['total_cycles_mean']:.0f} cyc ({s['total_us_mean']:.1f} us)")
    print(f"  {'phase':20s} {'mean lane':>10s} {'slowest':>10s} {'share':>6s}")
    for i, n in enumerate(NAMES):
        v = s["phases_cycles_mean"][n]
        print(f"  {n:20s} {res['mean_lane_step_phases'][n]:10.0f} {v:10.0f} {100 * v / s['total_cycles_mean']:5.1f}%")
    for k, v in s["solve_split_cycles_mean"].items():
        print(f"    solve: {k:16s} {v:10.0f} {100 * v / s['total_cycles_mean']:5.1f}%")
    if s["solve_bookkeeping_cycles_mean"]:
        for k, v in s["solve_bookkeeping_cycles_mean"].items():
            print(f"    solve: {k:16s} {v:10.0f} {100 * v / s['total_cycles_mean']:5.1f}%")
    t = s["toi_split_cycles_mean"]
    print(f"    TOI: scan + b2TimeOfImpact {t['scan_and_time_of_impact']:10.0f} (scan alone {s['toi_scan_alone_cycles_mean'] or 0:.0f}), "
          f"events {t['events']:10.0f}")
    c = s["collide_split_cycles_mean"]
    print(f"    collide: narrow phase {c['narrow_phase']:10.0f}, serial commit {c['serial_commit']:10.0f}")
    print(f"  slowest lane: island contacts {s['island_contacts_mean']:.2f}, velocity updates {s['velocity_updates_mean']:.0f}, "
          f"position passes {s['position_passes_mean']:.1f}, TOI events {s['toi_events_mean']:.2f}")
    if out:
        with open(out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
