"""Would splitting an island's velocity sweeps over two waves of one workgroup pay?  (analysis, CPU
only; VERDICT r4 item 5: the 3-block config runs one wave per SIMD at 1024 lanes, so a second wave
per world would use idle slots.)

    python tools/two_wave_model.py VELBENCH_TXT XCHBENCH_TXT [env] [lanes] [first_step] [last_step]

The oracle's work model (b2o_model_2wave, oracle/b2_oracle.c) replays every island's Gauss-Seidel
order with the device's exact sweep count and prices it (a) on one wave and (b) split over two waves
with the best contact partition: each wave keeps the sequential order of its contacts, a contact
waits for the previous update of each dynamic body it touches (+ one LDS handoff when that update
ran on the other wave), and both waves meet at every early-exit compare -- the only schedules that
keep the result bit-exact.  Update costs are one wave's measured cycles per contact update
(tools/velbench.py: by point count and by the number of contacts the wave holds: register paths
for 1-2, the lane-distributed path above); handoff and meeting costs are tools/micro/xchbench's
(flag and barrier).  The rest of each lane-step is priced as tools/chain_model.py does.  Printed:
the per-launch slowest lane-step, summed over the window, one wave vs two, for the measured handoff
and for cheaper hypothetical ones.
"""
from __future__ import annotations

import ctypes
import os
import re
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from gym_puzzles_amd.spawn import draw_bounds  # noqa: E402
from oracle.oracle import WORK_NAMES, batch_work, lib  # noqa: E402

C_POS, C_TOI, C_FIX, C_VEL = 850.0, 25000.0, 60000.0, 900.0   # tools/chain_model.py
W = {n: i for i, n in enumerate(WORK_NAMES)}


def velbench_costs(path: str) -> np.ndarray:
    """cost[(p - 1) * 8 + n - 1]: one-wave cycles per p-point contact update, n contacts on the wave."""
    med = {}
    for ln in open(path):
        m = re.match(r"blocks\s+1 nc (\d+) points (\d): cycles per contact update median\s+([\d.]+)", ln)
        if m and int(m.group(1)) < 100:
            med[(int(m.group(1)), int(m.group(2)))] = float(m.group(3))
    c = np.zeros(16)
    for p in (1, 2):
        for n in range(1, 9):
            q = min(n, 6)
            if (q, p) in med:
                v = med[(q, p)]
            elif q == 5 and (4, p) in med and (6, p) in med:
                v = 0.5 * (med[(4, p)] + med[(6, p)])
            else:   # 1-point costs not measured: the 2-point cost scaled by the one-contact ratio
                v = med[(q if q != 5 else 4, 2)] * med[(1, 1)] / med[(1, 2)]
            c[(p - 1) * 8 + n - 1] = v
    return c


def xch_costs(path: str) -> tuple[float, float]:
    flag = barrier = None
    for ln in open(path):
        m = re.match(r"(flag|barrier)\s+blocks\s+1: cycles per one-way handoff mean\s+([\d.]+)", ln)
        if m:
            if m.group(1) == "flag":
                flag = float(m.group(2))
            else:
                barrier = float(m.group(2))
    return flag, barrier


def main():
    cost = velbench_costs(sys.argv[1])
    x_meas, b_meas = xch_costs(sys.argv[2])
    env = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    lanes = int(sys.argv[4]) if len(sys.argv) > 4 else 1024
    s0 = int(sys.argv[5]) if len(sys.argv) > 5 else 6
    s1 = int(sys.argv[6]) if len(sys.argv) > 6 else 25
    L = lib()
    L.b2o_model_2wave.argtypes = [ctypes.c_void_p, ctypes.c_double, ctypes.c_double]
    print(f"env {env}, {lanes} lanes, steps {s0}-{s1} after spawn")
    print("cycles per contact update, 1 point (n = 1..8 on the wave):", " ".join(f"{v:.0f}" for v in cost[:8]))
    print("cycles per contact update, 2 points                       :", " ".join(f"{v:.0f}" for v in cost[8:]))
    print(f"measured handoff: flag {x_meas:.0f} cycles, barrier {b_meas:.0f} cycles (tools/micro/xchbench)")
    cbuf = (ctypes.c_double * 16)(*cost)
    for x in sorted({x_meas, 0.0, 100.0, 200.0, 400.0}):
        L.b2o_model_2wave(cbuf, x, b_meas)
        w = batch_work(env, lanes, s1, 17, draw_bounds(env), threads=os.cpu_count() or 1)[s0 - 1:s1]
        other = (C_FIX + C_POS * (w[..., W["pos_points"]] + w[..., W["toi_pos_points"]])
                 + C_VEL * w[..., W["toi_vel_upd"]] + C_TOI * (w[..., W["toi_vel_upd"]] > 0))
        one, two = other + w[..., W["vel_1wave"]], other + w[..., W["vel_2wave"]]
        m1, m2 = one.max(axis=1).sum(), two.max(axis=1).sum()
        vel_share = (w[..., W["vel_1wave"]][np.arange(w.shape[0]), one.argmax(axis=1)] / one.max(axis=1)).mean()
        tag = " (measured)" if x == x_meas else ""
        print(f"handoff {x:6.0f} cycles{tag}: slowest lane-steps one wave {m1 / 1e6:7.2f} Mcyc, two waves {m2 / 1e6:7.2f} Mcyc "
              f"(x{m1 / m2:.3f}); velocity share of the one-wave slowest lane-step {vel_share:.2f}; "
              f"all lanes' sweeps x{w[..., W['vel_1wave']].sum() / max(w[..., W['vel_2wave']].sum(), 1):.3f}")
    L.b2o_model_dual.argtypes = [ctypes.c_double, ctypes.c_int]
    for factor, window in ((1.0, -16), (1.0, 16), (1.1, 16), (1.2, 16)):   # paired updates on one wave: no handoff, each slot dearer
        L.b2o_model_2wave(cbuf, 0.0, 0.0)
        L.b2o_model_dual(factor, window)
        w = batch_work(env, lanes, s1, 17, draw_bounds(env), threads=os.cpu_count() or 1)[s0 - 1:s1]
        other = (C_FIX + C_POS * (w[..., W["pos_points"]] + w[..., W["toi_pos_points"]])
                 + C_VEL * w[..., W["toi_vel_upd"]] + C_TOI * (w[..., W["toi_vel_upd"]] > 0))
        one, two = other + w[..., W["vel_1wave"]], other + w[..., W["vel_2wave"]]
        m1, m2 = one.max(axis=1).sum(), two.max(axis=1).sum()
        print(f"paired lanes{' (no drains)' if window < 0 else ''}, slot = {factor:.1f} updates: slowest lane-steps one wave {m1 / 1e6:7.2f} Mcyc, paired {m2 / 1e6:7.2f} Mcyc "
              f"(x{m1 / m2:.3f}); all lanes' sweeps x{w[..., W['vel_1wave']].sum() / max(w[..., W['vel_2wave']].sum(), 1):.3f}")
    L.b2o_model_dual(0.0, 0)
    L.b2o_model_2wave(None, 0.0, 0.0)


if __name__ == "__main__":
    main()
