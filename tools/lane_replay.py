"""Contended vs standalone cost of the slowest lanes (diagnostic; -DMRP_STAMPS build):
    MRP_LIB=gym_puzzles_amd/libmrp_stamps.so python tools/lane_replay.py [env] [lanes] [warm] [n]
Steps a full batch, picks the n slowest lanes of one step, replays each of those lane-steps alone
(a one-lane batch holding the saved state, same RNG keys) and prints both phase traces."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from gym_puzzles_amd import Batch, _native  # noqa: E402

NAMES = "load act fnc0 coll solve fnc1 toi obs out reset store".split()


def trace(L, n):
    tr = np.zeros((n, _native.trace_words()), np.uint32)
    L.mrp_debug_trace(0, tr.ctypes.data_as(ctypes.c_void_p), n)
    return tr


def row(r):
    return (f"{r[11]:9d} | " + " ".join(f"{v:7d}" for v in r[:11]) + f" | nc {r[12]} toi {r[13]} pos {r[14]} vel {r[15]}"
            f" | vel {r[16]} pos {r[17]} pre {r[18]} maxisl {r[19]}"
            # words 20-23 are cycle splits since round 4 (mrp_world.h g_trace), not body pairs
            f" | toi scan {r[20]} events {r[21]} | collide narrow {r[22]} commit {r[23]}")


env = int(sys.argv[1]) if len(sys.argv) > 1 else 0
lanes = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
warm = int(sys.argv[3]) if len(sys.argv) > 3 else 10
n = int(sys.argv[4]) if len(sys.argv) > 4 else 6
L = _native.load()
b = Batch(env, lanes, seed=17)
b.set_auto_reset(True)
b.reset()
for _ in range(warm):
    b.step()
st = b.get_state()
b.step()
tr = trace(L, lanes)
order = np.argsort(-tr[:, 11].astype(np.int64))[:n]
print("phases:", " ".join(NAMES))
for l in order:
    print(f"lane {l:5d} in the batch: " + row(tr[l]), flush=True)
    one = Batch(env, 1, seed=17, lane_offset=int(l))
    one.set_auto_reset(True)
    one.set_state(st[l:l + 1])
    one.step()
    print(f"           alone:        " + row(trace(L, 1)[0]), flush=True)
    one.close()
