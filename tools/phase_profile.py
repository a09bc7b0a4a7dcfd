"""Per-phase time split of k_step (diagnostic build with -DMRP_STAMPS).
    python -m gym_puzzles_amd.build --stamps && MRP_LIB=gym_puzzles_amd/libmrp_stamps.so python tools/phase_profile.py
Thread 0 of each lane stamps s_memtime at phase boundaries; shares are of total lane time."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from gym_puzzles_amd import Batch, _native  # noqa: E402

NAMES = ["load+act", "apply_actions", "FNC(new fixtures)", "collide", "solve(islands)", "FNC(after solve)",
         "TOI", "obs/reward", "outputs", "auto-reset", "store"]


def main():
    env = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    lanes = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 100
    b = Batch(env, lanes, seed=17)
    b.set_auto_reset(True)
    b.reset()
    for _ in range(10):
        b.step()
    L = _native.load()
    buf = np.zeros(16, np.uint64)
    pmax, smax, rt = np.zeros(16, np.uint64), np.zeros(256, np.uint64), np.zeros(2, np.uint64)
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    L.mrp_debug_stamps(0, vp(buf))
    L.mrp_debug_stamps_ext(0, vp(pmax), vp(smax), vp(rt))
    for _ in range(steps):
        b.step()
    rc = L.mrp_debug_stamps(0, buf.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0, "not a -DMRP_STAMPS build"
    tot = buf[:11].astype(np.float64).sum()
    print(f"env {env} lanes {lanes} steps {steps}: mean thread-0 cycles per lane-step {tot / lanes / steps:.0f}")
    L.mrp_debug_stamps_ext(0, vp(pmax), vp(smax), vp(rt))
    ghz = 0.1 * rt[0] / max(rt[1], 1)   # s_memrealtime ticks at 100 MHz
    sm = smax[smax > 0].astype(np.float64)
    print(f"  s_memtime clock {ghz:.3f} GHz; mean lane total {rt[0] / lanes / steps:.0f} cyc; "
          f"slowest lane per step: mean {sm.mean():.0f} max {sm.max():.0f} cyc ({sm.mean() / ghz / 1e3:.1f} us mean)")
    for i, n in enumerate(NAMES):
        print(f"  {n:20s} {buf[i] / lanes / steps:10.0f} cyc  {100 * buf[i] / tot:5.1f}%   max {pmax[i]:10d}")
    tr = np.zeros((lanes, 24), np.uint32)
    L.mrp_debug_trace(0, vp(tr), lanes)
    order = np.argsort(-tr[:, 11].astype(np.int64))
    print("  last step, slowest lanes: total | load act fnc0 coll solve fnc1 toi obs out reset store | nc toi pos velunits")
    for l in order[:12]:
        r = tr[l]
        print(f"    lane {l:5d} {r[11]:9d} | " + " ".join(f"{v:7d}" for v in r[:11]) + f" | {r[12]:3d} {r[13]:3d} {r[14]:3d} {r[15]:4d}")
    print(f"  last step mean total {tr[:, 11].mean():.0f}; lanes with nc>0: {(tr[:, 12] > 0).mean():.3f}; "
          f"mean nc {tr[:, 12].mean():.2f}; toi>0: {(tr[:, 13] > 0).mean():.3f}")


if __name__ == "__main__":
    main()
