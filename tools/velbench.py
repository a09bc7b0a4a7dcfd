"""Single-wave and full-chip cost of one lane-distributed velocity contact update
(mrp_debug_velbench): python tools/velbench.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from gym_puzzles_amd import _native  # noqa: E402

L = _native.load()
iters = 180
for blocks in (1, 1024, 4096):
    # nc >= 100: a chain of nc - 100 contacts (contact i between bodies i and i + 1)
    for nc, pc in ((1, 1), (1, 2), (2, 2), (3, 2), (4, 2), (6, 2), (104, 2), (106, 2), (2, 1), (3, 1), (4, 1), (6, 1)):
        out = np.zeros(blocks, np.uint64)
        rc = L.mrp_debug_velbench(0, nc, pc, iters, blocks, out.ctypes.data)
        if rc != 0 and nc >= 100:
            print(f"blocks {blocks:5d} nc {nc}: not in this library", flush=True)
            continue
        assert rc == 0, rc
        L.mrp_debug_velbench(0, nc, pc, iters, blocks, out.ctypes.data)   # warm
        per = out.astype(np.float64) / (iters * (nc % 100))
        print(f"blocks {blocks:5d} nc {nc} points {pc}: cycles per contact update median {np.median(per):7.1f} max {per.max():7.1f}", flush=True)
