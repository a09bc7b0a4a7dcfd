"""Serial-chain model of k_step (analysis; CPU only): how long each launch's slowest lane takes,
from the oracle's work counts (oracle/b2_oracle.h OrWork: velocity sweeps counted with the
device's exact early exit, position point updates, TOI events), and how much of it grouping each
island's Gauss-Seidel order into dependency levels would remove.

    python tools/chain_model.py [env] [lanes] [first_step] [last_step] [kernel_trace.csv warmup]

Costs per unit are one wave's measured cycles (~900 cycles per velocity contact update,
~850 per position point update incl. its b2Rot::Set, ~25 K per TOI event, ~60 K of fixed per-step
work).  With a kernel trace of bench.py (tools/sessions/r3_session.sh) the model is set beside the measured
per-launch durations of the same steps.
"""
from __future__ import annotations

import csv
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from gym_puzzles_amd.spawn import draw_bounds  # noqa: E402
from oracle.oracle import WORK_NAMES, batch_work  # noqa: E402

C_VEL, C_POS, C_TOI, C_FIX = 900.0, 850.0, 25000.0, 60000.0
W = {n: i for i, n in enumerate(WORK_NAMES)}


def lane_cycles(w: np.ndarray, mode: str) -> np.ndarray:
    """[..., 16] work -> modelled cycles of the lane's serial chain.  mode: 'order' (contact by
    contact, as k_step runs it), 'levels' (dependency levels within each sweep / pass) or 'pipe'
    (the sweeps / passes unrolled: the critical path of the whole solve)."""
    if mode == "order":
        vel = w[..., W["vel_upd1"]] + w[..., W["vel_upd2"]] + w[..., W["toi_vel_upd"]]
        pos = w[..., W["pos_points"]] + w[..., W["toi_pos_points"]]
    elif mode == "levels":
        vel = w[..., W["vel_levels"]] + w[..., W["toi_vel_levels"]]
        pos = w[..., W["pos_level_points"]] + w[..., W["toi_pos_level_points"]]
    elif mode == "pipe":
        vel, pos = w[..., W["vel_pipe"]], w[..., W["pos_pipe"]]
    else:   # 'islands': contact order, but a step's independent islands solved concurrently
        vel = w[..., W["vel_upd1"]] + w[..., W["vel_upd2"]] + w[..., W["toi_vel_upd"]] - w[..., W["isl_concurrent_save"]]
        pos = w[..., W["pos_points"]] + w[..., W["toi_pos_points"]]
    return C_FIX + C_VEL * vel + C_POS * pos + C_TOI * (w[..., W["toi_vel_upd"]] > 0)


def main():
    env = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    lanes = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    s0 = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    s1 = int(sys.argv[4]) if len(sys.argv) > 4 else 25
    w = batch_work(env, lanes, s1, 17, draw_bounds(env), threads=os.cpu_count() or 1)
    if os.environ.get("MODEL_PERIOD"):   # what detecting velocity-sweep periods up to P would take off
        import ctypes
        from oracle.oracle import lib
        lib().b2o_model_period.argtypes = [ctypes.c_int]
        lib().b2o_model_period(int(os.environ["MODEL_PERIOD"]))
        wp = batch_work(env, lanes, s1, 17, draw_bounds(env), threads=os.cpu_count() or 1)[s0 - 1:s1]
        lib().b2o_model_period(0)
        a, b = lane_cycles(w[s0 - 1:s1], "order").max(axis=1).sum(), lane_cycles(wp, "order").max(axis=1).sum()
        print(f"period detection up to {os.environ['MODEL_PERIOD']}: slowest-lane sum {a / 1e6:.2f} -> {b / 1e6:.2f} Mcyc (x{a / b:.3f})")
    win = w[s0 - 1:s1]                      # step s (1-based after spawn) = row s - 1
    now, lev, pipe = lane_cycles(win, "order"), lane_cycles(win, "levels"), lane_cycles(win, "pipe")
    mx_now, mx_lev, mx_pipe = now.max(axis=1), lev.max(axis=1), pipe.max(axis=1)
    mx_isl = lane_cycles(win, "islands").max(axis=1)
    arg = now.argmax(axis=1)
    meas = None
    if len(sys.argv) > 6:
        rows = []
        with open(sys.argv[5]) as f:
            for r in csv.DictReader(f):
                if "k_step" in r["Kernel_Name"]:
                    rows.append((int(r["Dispatch_Id"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6))
        rows.sort()
        warm = int(sys.argv[6])
        meas = [d for _, d in rows[warm:warm + (s1 - s0 + 1)]]
    print(f"env {env}, {lanes} lanes, steps {s0}-{s1} after spawn")
    print("step  slowest-lane  vel-upd  vel-levels  pos-pts  pos-lvl-pts  model-Mcyc  levels-Mcyc" +
          ("  measured-ms" if meas else ""))
    for k in range(win.shape[0]):
        l = arg[k]
        x = win[k, l]
        line = (f"{s0 + k:4d}  {l:12d}  {x[W['vel_upd1']] + x[W['vel_upd2']] + x[W['toi_vel_upd']]:7d}  "
                f"{x[W['vel_levels']] + x[W['toi_vel_levels']]:10d}  {x[W['pos_points']] + x[W['toi_pos_points']]:7d}  "
                f"{x[W['pos_level_points']] + x[W['toi_pos_level_points']]:11d}  {mx_now[k] / 1e6:10.3f}  {mx_lev[k] / 1e6:11.3f}")
        if meas:
            line += f"  {meas[k]:11.4f}"
        print(line)
    print(f"sum of per-step slowest lanes: contact order {mx_now.sum() / 1e6:.2f} Mcyc, dependency levels "
          f"{mx_lev.sum() / 1e6:.2f} Mcyc (x{mx_now.sum() / mx_lev.sum():.3f}), unrolled critical path "
          f"{mx_pipe.sum() / 1e6:.2f} Mcyc (x{mx_now.sum() / mx_pipe.sum():.3f}), independent islands concurrent "
          f"{mx_isl.sum() / 1e6:.2f} Mcyc (x{mx_now.sum() / mx_isl.sum():.3f})")
    if meas:
        r = np.corrcoef(mx_now, np.array(meas))[0, 1]
        print(f"correlation of the modelled slowest lane with the measured launch time: {r:.3f}; "
              f"implied clock {mx_now.sum() / (sum(meas) * 1e-3) / 1e9:.2f} GHz")
    tot = win.sum(axis=(0, 1))
    v = tot[W["vel_upd1"]] + tot[W["vel_upd2"]] + tot[W["toi_vel_upd"]]
    print(f"all lanes: velocity updates {v}, levels {tot[W['vel_levels']] + tot[W['toi_vel_levels']]}, "
          f"position points {tot[W['pos_points']] + tot[W['toi_pos_points']]}, "
          f"level points {tot[W['pos_level_points']] + tot[W['toi_pos_level_points']]}, "
          f"unrolled velocity path {tot[W['vel_pipe']]}, position path {tot[W['pos_pipe']]}")


if __name__ == "__main__":
    main()
