"""Single-wave cost of one position-pass point update (mrp_debug_posbench): python tools/posbench.py

A synthetic island of nc static-wall contacts squeezing one block (walls alternately above and below
it, so the passes never reach the exit test, like the slowest v0 lanes' agent-block-wall islands);
the register paths solve 1-2 contacts, the lanes path 3 and more.  Cycles per point update =
cycles / (passes * nc * points)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from gym_puzzles_amd import _native  # noqa: E402

L = _native.load()
if not hasattr(L, "mrp_debug_posbench"):
    print("posbench: not in this library")
    sys.exit(0)
iters = 60
for blocks in (1, 1024):
    for nc, pc in ((1, 1), (1, 2), (2, 2), (3, 2), (4, 2), (3, 1)):
        out = np.zeros(2 * blocks, np.uint64)
        assert L.mrp_debug_posbench(0, nc, pc, iters, blocks, out.ctypes.data) == 0
        L.mrp_debug_posbench(0, nc, pc, iters, blocks, out.ctypes.data)   # warm
        cyc, passes = out[0::2].astype(np.float64), out[1::2].astype(np.float64)
        per = cyc / (passes * nc * pc)
        print(f"blocks {blocks:5d} nc {nc} points {pc}: passes {int(passes[0]):3d}  cycles per point update median "
              f"{np.median(per):7.1f} max {per.max():7.1f}", flush=True)
