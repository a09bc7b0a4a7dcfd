"""What slows the slowest lane down inside a batch (diagnostic; -DMRP_STAMPS build):
    MRP_LIB=gym_puzzles_amd/libmrp_stamps.so python tools/contention.py [env] [lanes] [warm]
Steps a full batch `warm` steps, then one step with host actions, and picks the slowest lane s.
Then re-runs that lane-step (same state, same action) beside different co-runners:
  K copies of s (K = 1 .. 8192), and s beside lanes-1 copies of the median lane / of the
  fastest lane / the original batch (s moved to workgroup 0),
printing s's phase split (total, island set-up, velocity sweeps, position passes) and the
s_memtime clock."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from gym_puzzles_amd import Batch, _native  # noqa: E402

TW = _native.trace_words()
vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731


def trace(L, n):
    tr = np.zeros((n, TW), np.uint32)
    L.mrp_debug_trace(0, vp(tr), n)
    return tr


def clock(L):
    pmax, smax, rt = np.zeros(16, np.uint64), np.zeros(256, np.uint64), np.zeros(2, np.uint64)
    L.mrp_debug_stamps_ext(0, vp(pmax), vp(smax), vp(rt))
    return 0.1 * rt[0] / max(rt[1], 1)


def run(L, env, states, acts, label):
    n = len(states)
    bk = Batch(env, n, seed=17)
    bk.set_auto_reset(True)
    bk.set_state(states)
    bk.step(acts)                    # warm the code path once
    bk.set_state(states)
    clock(L)
    bk.step(acts)
    t = trace(L, min(n, 16384))
    g = clock(L)
    r = t[0]
    print(f"{label:34s} clock {g:.2f} GHz | s: total {r[11]:8d} pre {r[18]:7d} vel {r[16]:7d} pos {r[17]:7d} "
          f"coll {r[3]:6d} toi {r[6]:6d} store {r[10]:6d} | all lanes: total max {t[:, 11].max():8d} median {int(np.median(t[:, 11])):7d}",
          flush=True)
    bk.close()


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
b.step(acts)
tr = trace(L, lanes)
ghz = clock(L)
order = np.argsort(-tr[:, 11].astype(np.int64))
s, m, f = order[0], order[lanes // 2], order[-1]
r = tr[s]
print(f"original batch {lanes}: clock {ghz:.2f} GHz, slowest lane {s}: total {r[11]} pre {r[18]} vel {r[16]} pos {r[17]} "
      f"nc {r[12]}; median lane {m} total {tr[m, 11]}; fastest lane {f} total {tr[f, 11]}", flush=True)
for K in (1, 64, 1024, 4096):
    run(L, env, np.repeat(st[s:s + 1], K, 0), np.repeat(acts[s:s + 1], K, 0), f"{K} copies of s")
for name, other in (("median", m), ("fastest", f)):
    sts = np.repeat(st[other:other + 1], lanes, 0)
    ac = np.repeat(acts[other:other + 1], lanes, 0)
    sts[0] = st[s]
    ac[0] = acts[s]
    run(L, env, sts, ac, f"s + {lanes - 1} x {name}")
perm = np.concatenate([[s], np.delete(np.arange(lanes), s)])
run(L, env, st[perm], acts[perm], "s + the original batch")
