"""Generate the committed golden fixtures under tests/golden/ (run from the repo root):

    python tests/golden/make_golden.py

1. ``spawn_draws.json`` -- reference-RNG inputs, pinned to numpy's frozen legacy streams:
   the values ``np.random.seed(s)`` + the reference's ``np.random.uniform`` calls produce at
   reset (multi_robot_puzzle_00.py:311-315,366-367; multi_robot_puzzle_02.py:307-308,324,
   358-359), and gym 0.21 ``action_space.seed(s)`` + ``sample()`` actions
   (gym_puzzles/tests/test_env.py:17-20,28), for seeds 0, 17 and 2021.
2. ``traj_env{E}.npz`` -- self-consistency trajectories of the CPU oracle (oracle/): 4 lanes x
   64 steps per env id with host-drawn spawns and actions (including masked resets of finished
   lanes).  Inputs and outputs are both stored; outputs are float32 as the C ABI returns them.
   These are NOT pybox2d-verified (parity vs pybox2d is unpinned); they pin the
   oracle against regressions and give the GPU path fixed expected values.
3. ``scenario_v0_seed17.npz`` -- the reference's own test flow (test_env.py:12-29) replayed for
   MultiRobotPuzzle-v0: env construction runs reset() once (multi_robot_puzzle_00.py:209) with
   whatever the global RNG holds (here: np.random.seed(0) before construction), then
   np.random.seed(17), action_space.seed(17), reset(), and 200 steps of action_space.sample().
4. ``scenario_v3heavy_seed17.npz`` -- the same test file's actual target, MultiRobotPuzzle-v3 with
   heavy=True (test_env.py:12-36): two resets, then steps until done or the 1500-step TimeLimit.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from gym_puzzles_amd.seeding import Box  # noqa: E402
from gym_puzzles_amd.spawn import reference_draws  # noqa: E402
from oracle.oracle import OracleEnv  # noqa: E402

LANES, STEPS = 4, 64


def spawn_fixture():
    out = {}
    for env_id in range(7):
        for seed in (0, 17, 2021):
            np.random.seed(seed)
            d = reference_draws(env_id)          # global np.random, like the reference
            out[f"draws/{env_id}/{seed}"] = [float(v) for v in d]
    for act_dim in (4, 6, 15):
        for seed in (0, 17, 2021):
            sp = Box(-1.0, 1.0, shape=(act_dim,))
            sp.seed(seed)
            out[f"actions/{act_dim}/{seed}"] = [[float(v) for v in sp.sample()] for _ in range(3)]
    with open(os.path.join(HERE, "spawn_draws.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


def trajectory(env_id: int):
    rs = np.random.RandomState(100 + env_id)
    orc = [OracleEnv(env_id) for _ in range(LANES)]
    A, D = orc[0].act_dim, orc[0].n_draws
    draws0 = np.stack([reference_draws(env_id, rs) for _ in range(LANES)])
    act0 = rs.uniform(-1, 1, size=(LANES, A)).astype(np.float32)
    obs0 = np.stack([o.reset(draws0[l], act0[l]) for l, o in enumerate(orc)]).astype(np.float32)
    acts = np.zeros((STEPS, LANES, A), np.float32)
    obs = np.zeros((STEPS, LANES, orc[0].obs_dim), np.float32)
    rew = np.zeros((STEPS, LANES), np.float32)
    done = np.zeros((STEPS, LANES), np.uint8)
    bodies = np.zeros((STEPS, LANES, 6 * (orc[0].n_agents + orc[0].n_blocks)), np.float32)
    rdraws = np.zeros((STEPS, LANES, D), np.float64)       # reset inputs for lanes done at step t
    racts = np.zeros((STEPS, LANES, A), np.float32)
    robs = np.zeros((STEPS, LANES, orc[0].obs_dim), np.float32)
    for t in range(STEPS):
        acts[t] = rs.uniform(-1, 1, size=(LANES, A)).astype(np.float32)
        for l, o in enumerate(orc):
            ob, r, d, _ = o.step(acts[t, l])
            obs[t, l], rew[t, l], done[t, l] = ob, r, d
            bodies[t, l] = o.bodies()
            if d:
                rdraws[t, l] = reference_draws(env_id, rs)
                racts[t, l] = rs.uniform(-1, 1, size=A).astype(np.float32)
                robs[t, l] = o.reset(rdraws[t, l], racts[t, l])
    np.savez_compressed(os.path.join(HERE, f"traj_env{env_id}.npz"), draws0=draws0, act0=act0, obs0=obs0,
                        acts=acts, obs=obs, reward=rew, done=done, bodies=bodies, rdraws=rdraws, racts=racts,
                        robs=robs)


def scenario_v0():
    env_id, steps = 0, 200
    o = OracleEnv(env_id)
    sp = Box(-1.0, 1.0, shape=(o.act_dim,))
    np.random.seed(0)                                  # whatever the process held before seeding
    o.reset(reference_draws(env_id), sp.sample())      # __init__ -> self.reset()  (:209)
    np.random.seed(17)
    sp.seed(17)
    draws = reference_draws(env_id)
    a0 = sp.sample()
    obs0 = o.reset(draws, a0).astype(np.float32)
    acts = np.zeros((steps, o.act_dim), np.float32)
    obs = np.zeros((steps, o.obs_dim), np.float32)
    rew = np.zeros(steps, np.float64)
    for t in range(steps):
        acts[t] = sp.sample()
        ob, r, d, _ = o.step(acts[t])
        obs[t], rew[t] = ob, r
        assert not d
    np.savez_compressed(os.path.join(HERE, "scenario_v0_seed17.npz"), draws=draws, act0=a0, obs0=obs0, acts=acts,
                        obs=obs, reward=rew, bodies=o.bodies())


def scenario_v3_heavy():
    """gym_puzzles/tests/test_env.py itself: gym.make('MultiRobotPuzzle-v3', heavy=True) (the
    constructor's reset() draws from whatever the global RNG holds -- np.random.seed(0) here),
    np.random.seed(17), env.seed(17), action_space.seed(17), obs = env.reset(), then for the first
    of its 5 episodes env.reset() and action_space.sample() steps until done (TimeLimit 1500;
    `done` is never cleared, so the later episodes run no steps)."""
    env_id, limit = 6, 1500
    o = OracleEnv(env_id)
    sp = Box(-1.0, 1.0, shape=(o.act_dim,))
    np.random.seed(0)
    o.reset(reference_draws(env_id), sp.sample())
    np.random.seed(17)
    sp.seed(17)
    d1 = reference_draws(env_id)
    a1 = sp.sample()
    obs1 = o.reset(d1, a1).astype(np.float32)
    d2 = reference_draws(env_id)
    a2 = sp.sample()
    obs2 = o.reset(d2, a2).astype(np.float32)
    acts, obs, rew, done = [], [], [], []
    for t in range(limit):
        a = sp.sample()
        ob, r, dn, _ = o.step(a)
        acts.append(a); obs.append(ob.astype(np.float32)); rew.append(r); done.append(dn)
        if dn:
            break
    np.savez_compressed(os.path.join(HERE, "scenario_v3heavy_seed17.npz"), draws=np.stack([d1, d2]),
                        act0=np.stack([a1, a2]), obs0=np.stack([obs1, obs2]), acts=np.array(acts, np.float32),
                        obs=np.array(obs, np.float32), reward=np.array(rew, np.float64),
                        done=np.array(done, np.uint8), bodies=o.bodies())


if __name__ == "__main__":
    spawn_fixture()
    for e in range(7):
        trajectory(e)
    scenario_v0()
    scenario_v3_heavy()
    print("golden fixtures written to", HERE)
