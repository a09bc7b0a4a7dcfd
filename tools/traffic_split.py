"""Where a k_step launch's HBM bytes go, by part of the lane state (diagnostic, GPU box):

    python tools/traffic_split.py ENV LANES [WARMUP STEPS OUT.json]

k_step moves each lane's LaneState<ENV> between HBM and LDS once per launch (mrp_lane.h StateIO):
every word outside the contact-slot arrays in 16-B granules, and the contact-slot arrays only below
the lane's high-water mark cHW (word by word, or in 16-B granules for the units built with
MRP_CONTACT_GRANULES).  This replays bench.py's window (device-RNG actions, auto-reset) and reads
every lane's cHW before and after each timed launch (mrp_get_state), so the bytes each part of the
state moves are counted exactly as StateIO moves them; the outputs (obs, reward, done / truncated /
status) are added.  What PMC traffic (profiles/pmc_traffic.json, FETCH_SIZE x 2 + WRITE_SIZE) shows
beyond this sum is what the state round trip does not explain: constant-table reads for the LDS
tables, scratch (spills), instruction fetch.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from lane_layout import fields, offsets  # noqa: E402

GRANULE_UNITS = {2, 3}   # build.py: MRP_CONTACT_GRANULES=1 on the v2 unit(s)
CONTACT = ("cnext", "cprev", "cfa", "cfb", "cflags", "ctoiCount", "ctoi", "cfric", "mpc", "mtype",
           "mlnx", "mlny", "mlpx", "mlpy", "mpx", "mpy", "mni", "mti", "mid")
PARTS = {
    "bodies": ("xpx", "xpy", "xs", "xc", "c0x", "c0y", "cx", "cy", "a0", "a", "alpha0", "vx", "vy", "w", "fx", "fy", "tq"),
    "broad_phase_tree": ("proxy", "tlx", "tly", "thx", "thy", "tpar", "tc1", "tc2", "th", "tud", "root", "freeList",
                         "nodeCount", "moveCount", "moveBuf"),
    "contact_list_heads": ("cHead", "cFree", "cCount", "cHW"),
}


def main():
    env = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    lanes = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    warmup = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    out = sys.argv[5] if len(sys.argv) > 5 else None
    from gym_puzzles_amd import Batch
    off, nw = offsets(env)
    f, nd, na, nb = fields(env)
    size = dict(f)
    c = size["cnext"]
    ncw = sum(size[n] for n in CONTACT)          # contact-slot words: NCA arrays of C words
    nca = ncw // c
    other = nw - ncw                             # moved whole, in 16-B granules
    b = Batch(env, lanes, seed=17)
    b.set_auto_reset(True)
    b.reset()
    for _ in range(warmup):
        b.step()
    O = b.obs_dim
    hw_in, hw_out = [], []
    for _ in range(steps):
        hw_in.append(b.get_state()[:, off["cHW"]].astype(np.int64).copy())
        b.step()
        hw_out.append(b.get_state()[:, off["cHW"]].astype(np.int64).copy())
    b.close()
    hin, hout = np.array(hw_in), np.array(hw_out)
    if env in GRANULE_UNITS:   # granules with any live word: about ceil over the slot runs; bound by whole words
        live_load = np.minimum(nca * ((hin + 3) // 4 * 4), ncw)
        live_store = np.minimum(nca * ((np.maximum(hin, hout) + 3) // 4 * 4), ncw)
    else:
        live_load = nca * hin
        live_store = nca * np.maximum(hin, hout)
    per_launch = lambda words: float(words.sum(axis=1).mean()) * 4.0   # noqa: E731  bytes per launch
    parts = {}
    for name, members in PARTS.items():
        w = sum(size[m] for m in members)
        parts[name] = 2.0 * w * 4 * lanes                  # read + written
    rest = other - sum(sum(size[m] for m in members) for members in PARTS.values())
    parts["env_layer_and_counters"] = 2.0 * rest * 4 * lanes
    parts["contact_slots_read"] = per_launch(live_load)
    parts["contact_slots_written"] = per_launch(live_store)
    parts["outputs"] = float(lanes * (4 * O + 4 + 3))
    total = sum(parts.values())
    res = {"env": env, "lanes": lanes, "timed_steps_after_spawn": [warmup + 1, warmup + steps],
           "lane_state_bytes": nw * 4, "contact_slot_words": ncw, "contact_arrays": nca, "contact_slots": c,
           "mean_cHW": float(hin.mean()), "max_cHW": int(hin.max()),
           "bytes_per_launch": parts, "state_round_trip_and_outputs_per_launch": total}
    print(f"env {env} lanes {lanes} steps {warmup + 1}-{warmup + steps}: LaneState {nw * 4} B, contact slots "
          f"{nca} x {c} words, mean cHW {hin.mean():.2f} (max {hin.max()})")
    for k, v in parts.items():
        print(f"  {k:28s} {v / 1e6:8.2f} MB per launch  ({100 * v / total:5.1f} %)")
    print(f"  {'total':28s} {total / 1e6:8.2f} MB per launch")
    if out:
        with open(out, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
