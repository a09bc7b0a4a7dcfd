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
    L.mrp_debug_stamps(0, buf.ctypes.data_as(ctypes.c_void_p))
    for _ in range(steps):
        b.step()
    rc = L.mrp_debug_stamps(0, buf.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0, "not a -DMRP_STAMPS build"
    tot = buf[:11].astype(np.float64).sum()
    print(f"env {env} lanes {lanes} steps {steps}: mean thread-0 cycles per lane-step {tot / lanes / steps:.0f}")
    for i, n in enumerate(NAMES):
        print(f"  {n:20s} {buf[i] / lanes / steps:10.0f} cyc  {100 * buf[i] / tot:5.1f}%")


if __name__ == "__main__":
    main()
