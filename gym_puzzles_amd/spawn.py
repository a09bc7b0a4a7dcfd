"""Host-side spawn draws in the reference's order (the reference draws from numpy's
*global* ``np.random``, not ``self.np_random``).

``reference_draws(env_id, rs)`` returns exactly the float64 values the reference's
``np.random.uniform(low, high)`` calls produce, in call order:

* v0 / Heavy-v0 (``multi_robot_puzzle_00.py:311-315,366-367``): block x, y, angle, then
  x, y per agent.
* v2 / Heavy-v2 (``multi_robot_puzzle_02.py:324,358-359,307-308``): block angle, then x, y
  per agent, then goal x, y (``_set_random_goal``; SIMPLE=True places the block at the
  screen centre and fixes agent heading at 3/2*pi).
* 3-block (build-defined): one angle per block (T, L, I), agents, goal.
* v3 / v3 heavy (``core.py:212-215,231-232``): block x, y, angle, then x, y per agent.
"""
from __future__ import annotations

import numpy as np

# v0 constants (multi_robot_puzzle_00.py:38-43)
_V0_SCALE, _V0_W, _V0_H, _V0_BORDER = 30.0, 640, 480, 1
# v2 constants (multi_robot_puzzle_02.py:39-44, 305)
_V2_SCALE, _V2_W, _V2_H, _V2_BORDER, _V2_GOAL_BORDER = 140.0 * 4, 1440, 810, 0.3, 0.4

# v3 constants (core.py:16-19, 97-98)
_V3_SCALE, _V3_W, _V3_H, _V3_BORDER = 30.0, 640, 480, 1

# env id -> (version, agents, blocks, heavy) (csrc/mrp_config.h ENV_CFG); ids 7-10 / 11-14 are
# MultiRobotPuzzle2 / MultiRobotPuzzleHeavy2 constructed with num_agents = 1, 3, 4, 5, ids 15-18 /
# 19-22 RobotPuzzleBase(num_agents = 1, 3, 4, 5) with heavy False / True
ENV_CFG = {0: (0, 2, 1, 0), 1: (0, 5, 1, 1), 2: (2, 2, 1, 0), 3: (2, 2, 1, 1), 4: (2, 2, 3, 1), 5: (3, 2, 1, 0), 6: (3, 2, 1, 1),
           7: (2, 1, 1, 0), 8: (2, 3, 1, 0), 9: (2, 4, 1, 0), 10: (2, 5, 1, 0),
           11: (2, 1, 1, 1), 12: (2, 3, 1, 1), 13: (2, 4, 1, 1), 14: (2, 5, 1, 1),
           15: (3, 1, 1, 0), 16: (3, 3, 1, 0), 17: (3, 4, 1, 0), 18: (3, 5, 1, 0),
           19: (3, 1, 1, 1), 20: (3, 3, 1, 1), 21: (3, 4, 1, 1), 22: (3, 5, 1, 1)}
ENV_VERSION = {e: c[0] for e, c in ENV_CFG.items()}
N_AGENTS = {e: c[1] for e, c in ENV_CFG.items()}
N_BLOCKS = {e: c[2] for e, c in ENV_CFG.items()}
# MultiRobotPuzzle2(num_agents=N) / MultiRobotPuzzleHeavy2(num_agents=N) -> env id
V2_AGENT_IDS = {(c[3], c[1]): e for e, c in ENV_CFG.items() if c[0] == 2 and c[2] == 1}
# RobotPuzzleBase(num_agents=N, heavy=h) -> env id
V3_AGENT_IDS = {(c[3], c[1]): e for e, c in ENV_CFG.items() if c[0] == 3}


def draw_bounds(env_id: int):
    """(low, high) of every uniform draw of one reset, in call order."""
    b = []
    if ENV_VERSION[env_id] == 0:
        xr = (_V0_BORDER, _V0_W / _V0_SCALE - _V0_BORDER)
        yr = (_V0_BORDER, _V0_H / _V0_SCALE - _V0_BORDER)
        b += [xr, yr, (0, 2 * np.pi)]
        b += [xr, yr] * N_AGENTS[env_id]
    elif ENV_VERSION[env_id] == 3:
        b += [(_V3_W / _V3_SCALE / 3 + 2 * _V3_BORDER, _V3_W / _V3_SCALE * 2 / 3 - 2 * _V3_BORDER),
              (3 * _V3_BORDER, _V3_H / _V3_SCALE - 3 * _V3_BORDER), (0, 2 * np.pi)]
        b += [(_V3_BORDER, _V3_W / _V3_SCALE / 3 - 2 * _V3_BORDER), (_V3_BORDER, _V3_H / _V3_SCALE - _V3_BORDER)] * N_AGENTS[env_id]
    else:
        b += [(0, 2 * np.pi)] * N_BLOCKS[env_id]
        xr = (_V2_BORDER, _V2_W / _V2_SCALE / 3 - _V2_BORDER)
        yr = (_V2_BORDER, _V2_H / _V2_SCALE - _V2_BORDER)
        b += [xr, yr] * N_AGENTS[env_id]
        b += [(_V2_W / _V2_SCALE * 2 / 3 + _V2_GOAL_BORDER, _V2_W / _V2_SCALE - _V2_GOAL_BORDER),
              (_V2_GOAL_BORDER, _V2_H / _V2_SCALE - _V2_GOAL_BORDER)]
    return b


def reference_draws(env_id: int, rs=None) -> np.ndarray:
    """Draw one reset's spawn values from ``rs`` (a RandomState; default: global np.random)."""
    rs = np.random if rs is None else rs
    return np.array([rs.uniform(lo, hi) for lo, hi in draw_bounds(env_id)], dtype=np.float64)


def sample_action(act_dim: int, rs) -> np.ndarray:
    """gym 0.21 ``Box.sample()`` for a bounded [-1, 1] box: uniform(low, high).astype(float32)."""
    return rs.uniform(low=-np.ones(act_dim), high=np.ones(act_dim), size=(act_dim,)).astype(np.float32)
