"""Replay captured lane-steps alone, one 1-lane k_step launch each (diagnostic, GPU box).

    python tools/issue_replay.py CAPTURE.npz OUT.json [REPEAT]

Each row of tools/issue_capture.py's file is stepped by a 1-lane batch holding the saved state
(same seed, global lane, step counter, so the same lane-step bit for bit).  Run it under
`rocprofv3 --pmc SQ_INSTS ...` for the instruction counts of exactly those lane-steps, under
`--kernel-trace` for their lone-wave durations, or with MRP_LIB=<stamps library> for their phase
split alone (written to OUT.json).  REPEAT (default 1) replays each row that many times.
"""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from gym_puzzles_amd import Batch, _native  # noqa: E402


def main():
    cap = np.load(sys.argv[1])
    out = sys.argv[2]
    repeat = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    env = int(cap["env"])
    L = _native.load()
    tr = np.zeros((1, _native.trace_words()), np.uint32)
    rows = []
    for k in range(len(cap["lane"])):
        lane = int(cap["lane"][k])
        for r in range(repeat):
            one = Batch(env, 1, seed=17, lane_offset=lane)
            one.set_auto_reset(True)
            one.set_state(cap["state"][k][None])
            one.step()
            have = L.mrp_debug_trace(0, tr.ctypes.data_as(ctypes.c_void_p), 1) == 0
            rows.append({"row": k, "lane": lane, "repeat": r, "trace_alone": tr[0].tolist() if have else None,
                         "trace_in_batch": cap["trace"][k].tolist()})
            one.close()
    with open(out, "w") as f:
        json.dump({"env": env, "rows": rows}, f)
    print(f"replayed {len(rows)} lane-steps of env {env}")


if __name__ == "__main__":
    main()
