"""Capture the lane-steps that set each launch's duration (diagnostic; -DMRP_STAMPS library).

    MRP_LIB=gym_puzzles_amd/libmrp_stamps.so python tools/issue_capture.py ENV LANES WARMUP STEPS OUT.npz

Runs bench.py's workload (seed 17, device-RNG actions, auto-reset), and for each of the STEPS timed
launches keeps the pre-step lane state of that launch's slowest lane (by the in-kernel s_memtime
total of the stamps build) with its phase trace, so tools/issue_replay.py can step exactly that
lane-step alone under rocprofv3 counters.  A lane's step is a pure function of its state and its
RNG keys (seed, global lane, step counter), so the replay is the same lane-step, bit for bit.
"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from gym_puzzles_amd import Batch, _native  # noqa: E402


def main():
    env, lanes, warmup, steps, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
    b = Batch(env, lanes, seed=17)
    b.set_auto_reset(True)
    b.reset()
    for _ in range(warmup):
        b.step()
    L = _native.load()
    tr = np.zeros((lanes, _native.trace_words()), np.uint32)
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    states, lanes_, traces, totals = [], [], [], []
    for _ in range(steps):
        st = b.get_state()
        b.step()
        assert L.mrp_debug_trace(0, vp(tr), lanes) == 0, "not a -DMRP_STAMPS build"
        tot = tr[:, 11].astype(np.int64)
        l = int(np.argmax(tot))
        states.append(st[l].copy())
        lanes_.append(l)
        traces.append(tr[l].copy())
        totals.append(np.sort(tot)[::-1][:16])
    np.savez(out, env=env, lanes=lanes, warmup=warmup, steps=steps, state=np.array(states), lane=np.array(lanes_),
             trace=np.array(traces), top16=np.array(totals))
    print(f"env {env}: captured {steps} slowest lane-steps (lanes {sorted(set(lanes_))[:12]}...), "
          f"mean in-batch total {np.mean([t[11] for t in traces]):.0f} cycles")


if __name__ == "__main__":
    main()
