"""How a slow lane's step time grows with the number of co-running copies (diagnostic; -DMRP_STAMPS build):
    MRP_LIB=gym_puzzles_amd/libmrp_stamps.so python tools/contention.py [env] [lanes] [warm]
Steps a full batch `warm` steps, then one step with host actions; picks the slowest lane and re-runs
that lane-step as K identical copies (same state, same action) for growing K, printing the mean and
max per-lane s_memtime totals, the s_memtime clock and the wall time of the launch."""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from gym_puzzles_amd import Batch, _native  # noqa: E402

vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731


def trace(L, n):
    tr = np.zeros((n, 16), np.uint32)
    L.mrp_debug_trace(0, vp(tr), n)
    return tr


def clock(L):
    pmax, smax, rt = np.zeros(16, np.uint64), np.zeros(256, np.uint64), np.zeros(2, np.uint64)
    L.mrp_debug_stamps_ext(0, vp(pmax), vp(smax), vp(rt))
    return 0.1 * rt[0] / max(rt[1], 1)


env = int(sys.argv[1]) if len(sys.argv) > 1 else 0
lanes = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
warm = int(sys.argv[3]) if len(sys.argv) > 3 else 8
L = _native.load()
b = Batch(env, lanes, seed=17)
b.set_auto_reset(True)
b.reset()
for _ in range(warm):
    b.step()
st = b.get_state()
rng = np.random.default_rng(5)
acts = rng.uniform(-1, 1, (lanes, b.act_dim)).astype(np.float32)
clock(L)
t0 = time.perf_counter()
b.step(acts)
wall = time.perf_counter() - t0
tr = trace(L, lanes)
ghz = clock(L)
order = np.argsort(-tr[:, 11].astype(np.int64))
s = order[0]
print(f"full batch {lanes}: wall {wall * 1e3:.3f} ms, clock {ghz:.2f} GHz, slowest lane {s}: total {tr[s, 11]} solve {tr[s, 4]} "
      f"nc {tr[s, 12]} pos {tr[s, 14]} vel {tr[s, 15]}; 2nd {tr[order[1], 11]}, 10th {tr[order[9], 11]}, median {int(np.median(tr[:, 11]))}",
      flush=True)
for K in (1, 2, 8, 64, 256, 512, 1024, 2048, 4096, 8192):
    bk = Batch(env, K, seed=17)
    bk.set_auto_reset(True)
    bk.set_state(np.repeat(st[s:s + 1], K, 0))
    a = np.repeat(acts[s:s + 1], K, 0)
    bk.step(a)                       # warm the code path once
    bk.set_state(np.repeat(st[s:s + 1], K, 0))
    clock(L)
    t0 = time.perf_counter()
    bk.step(a)
    wall = time.perf_counter() - t0
    t = trace(L, min(K, 16384))
    g = clock(L)
    tot = t[:, 11].astype(np.float64)
    print(f"K {K:5d}: wall {wall * 1e3:7.3f} ms  clock {g:.2f} GHz  lane total mean {tot.mean():9.0f} max {tot.max():9.0f} "
          f"solve mean {t[:, 4].mean():9.0f}", flush=True)
    bk.close()
