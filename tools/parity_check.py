"""GPU (libmrp) vs CPU oracle parity sweep: same spawn draws and actions, compare every
step bit for bit (obs, reward, done, body state).  Usage:
    python tools/parity_check.py --env 0 --lanes 64 --steps 300
Exit code 1 on the first mismatch (prints the lane/step/field)."""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from gym_puzzles_amd import Batch  # noqa: E402
from gym_puzzles_amd.spawn import reference_draws, sample_action  # noqa: E402
from oracle.oracle import OracleEnv  # noqa: E402


def run(env_id: int, lanes: int, steps: int, seed: int = 17, verbose: bool = True) -> int:
    rs_draw = [np.random.RandomState(seed + l) for l in range(lanes)]
    rs_act = np.random.RandomState(1000 + seed)
    b = Batch(env_id, lanes)
    draws = np.stack([reference_draws(env_id, r) for r in rs_draw])
    acts = rs_act.uniform(-1, 1, size=(lanes, b.act_dim)).astype(np.float32)
    orc = [OracleEnv(env_id) for _ in range(lanes)]
    t0 = time.time()
    obs = b.reset(draws, acts).copy()
    oobs = np.stack([o.reset(draws[l], acts[l]) for l, o in enumerate(orc)]).astype(np.float32)
    bad = 0

    def cmp(name, g, c, t):
        nonlocal bad
        g = np.asarray(g); c = np.asarray(c)
        diff = ~((g == c) | (np.isnan(g) & np.isnan(c)))
        if diff.any():
            idx = np.argwhere(diff)[0]
            print(f"MISMATCH env {env_id} step {t} {name} at {tuple(idx)}: gpu {g[tuple(idx)]!r} oracle {c[tuple(idx)]!r}"
                  f" ({int(diff.sum())} elements)", flush=True)
            bad += 1
            return False
        return True

    if not (cmp("reset_obs", obs, oobs, -1) & cmp("reset_bodies", b.bodies(), np.stack([o.bodies() for o in orc]), -1)):
        return 1
    for t in range(steps):
        a = rs_act.uniform(-1, 1, size=(lanes, b.act_dim)).astype(np.float32)
        obs, rew, done, trunc = b.step(a)
        res = [o.step(a[l]) for l, o in enumerate(orc)]
        oobs = np.stack([r[0] for r in res]).astype(np.float32)
        orew = np.array([r[1] for r in res]).astype(np.float32)
        odone = np.array([r[2] for r in res], np.uint8)
        ok = cmp("obs", obs, oobs, t) & cmp("reward", rew, orew, t) & cmp("done", done, odone, t)
        ok &= cmp("bodies", b.bodies(), np.stack([o.bodies() for o in orc]), t)
        if not ok:
            return 1
        # reset finished lanes the same way on both sides (host draws)
        fin = done.astype(bool) | trunc.astype(bool)
        if fin.any():
            d2 = np.stack([reference_draws(env_id, rs_draw[l]) for l in range(lanes)])
            a2 = rs_act.uniform(-1, 1, size=(lanes, b.act_dim)).astype(np.float32)
            obs2 = b.reset(d2, a2, mask=fin).copy()
            for l in np.nonzero(fin)[0]:
                o2 = orc[l].reset(d2[l], a2[l]).astype(np.float32)
                if not cmp("reset_obs", obs2[l], o2, t):
                    return 1
    toi = b.counters()
    if verbose:
        print(f"env {env_id}: {lanes} lanes x {steps} steps bitwise equal (gpu toi/pos counters {toi}) "
              f"[{time.time() - t0:.1f}s]", flush=True)
    return 0


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", type=int, nargs="+", default=[0])
    ap.add_argument("--lanes", type=int, default=64)
    ap.add_argument("--steps", type=int, default=300)
    args = ap.parse_args()
    rc = 0
    for e in args.env:
        rc |= run(e, args.lanes, args.steps)
    sys.exit(rc)
