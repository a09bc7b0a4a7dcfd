"""Diagnostic: first divergence between the device step and the oracle for given env ids.

For each env id: 64 lanes of host-input steps (as tests/test_gpu.py test_step_parity_host_inputs);
at the first step whose obs or bodies differ, print the lane, the step, the differing body
quantities and the lane's contact / island summary from the oracle, then continue with the next id.

    python tools/variant_diff.py 7 8 9 10
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from gym_puzzles_amd import Batch  # noqa: E402
from gym_puzzles_amd.spawn import reference_draws  # noqa: E402
from oracle import oracle  # noqa: E402


def run(env_id: int, lanes: int = 64, steps: int = 200) -> None:
    rs_d = [np.random.RandomState(17 + l) for l in range(lanes)]
    rs_a = np.random.RandomState(1017)
    b = Batch(env_id, lanes)
    envs = [oracle.OracleEnv(env_id) for _ in range(lanes)]
    draws = np.stack([reference_draws(env_id, r) for r in rs_d])
    acts = rs_a.uniform(-1, 1, size=(lanes, b.act_dim)).astype(np.float32)
    g = b.reset(draws, acts)
    c = np.stack([o.reset(draws[l], acts[l]) for l, o in enumerate(envs)]).astype(np.float32)
    if not np.array_equal(g, c):
        print(f"env {env_id}: reset obs differ in lanes {np.nonzero((g != c).any(1))[0].tolist()}")
        return
    prev_g = b.bodies().copy()
    for t in range(steps):
        a = rs_a.uniform(-1, 1, size=(lanes, b.act_dim)).astype(np.float32)
        obs, rew, done, _ = b.step(a)
        res = [o.step(a[l]) for l, o in enumerate(envs)]
        bg = b.bodies()
        bc = np.stack([o.bodies() for o in envs])
        bad = ~((bg == bc) | (np.isnan(bg) & np.isnan(bc)))
        if bad.any():
            lanes_bad = np.nonzero(bad.any(1))[0]
            l = int(lanes_bad[0])
            nd = bg.shape[1] // 6
            print(f"env {env_id}: step {t}: {len(lanes_bad)} lanes differ (first {l}); toi/pos counters gpu {b.counters()}")
            for k in np.nonzero(bad[l])[0]:
                print(f"   body {k // 6} q{k % 6}: gpu {bg[l, k]!r} oracle {bc[l, k]!r} (prev gpu {prev_g[l, k]!r})")
            print(f"   nd {nd}, flags gpu {b.flags()[l].tolist()}")
            return
        prev_g = bg.copy()
        if done.any():
            m = done.astype(bool)
            nd_ = np.stack([reference_draws(env_id, rs_d[l]) for l in range(lanes)])
            na = rs_a.uniform(-1, 1, size=(lanes, b.act_dim)).astype(np.float32)
            b.reset(nd_, na, mask=m)
            for l in np.nonzero(m)[0]:
                envs[l].reset(nd_[l], na[l])
    print(f"env {env_id}: {steps} steps x {lanes} lanes bitwise")


if __name__ == "__main__":
    for e in (int(x) for x in sys.argv[1:] or range(7, 15)):
        run(e)
