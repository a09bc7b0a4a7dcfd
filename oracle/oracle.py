"""TEST INFRASTRUCTURE ONLY -- ctypes front end of the CPU parity oracle.

Loads ``oracle/build/libmrp_oracle.so`` (plain-C restatement of the gym_puzzles step path
and the Box2D v2.3 subset it calls; see ``oracle/b2_oracle.h``).  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this module;
the product (``gym_puzzles_amd``) never does.

Parity of this oracle against pybox2d is UNPINNED: the reference's own tests pin no step
result and box2d-py is not importable in this image (SURVEY.md sections 4, 8c).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libmrp_oracle.so")
# solver variants of the same sources (oracle/Makefile): the checker carries the work model; the
# CPU baseline of bench.py times "port" (all 180 velocity sweeps, as b2Island::Solve runs them) and
# "early" (the device's exact period-1/2 early exit of the sweeps); all three give the same bits
VARIANTS = {"checker": _LIB_PATH, "port": os.path.join(_HERE, "build", "libmrp_oracle_port.so"),
            "early": os.path.join(_HERE, "build", "libmrp_oracle_early.so")}
_lib = None
_variants = {}

ENV_IDS = {
    "MultiRobotPuzzle-v0": 0,
    "MultiRobotPuzzleHeavy-v0": 1,
    "MultiRobotPuzzle-v2": 2,
    "MultiRobotPuzzleHeavy-v2": 3,
    "MultiRobotPuzzleHeavy-v2-3block": 4,
    "MultiRobotPuzzle-v3": 5,
    "MultiRobotPuzzle-v3-heavy": 6,
    "MultiRobotPuzzle-v2-agents1": 7, "MultiRobotPuzzle-v2-agents3": 8, "MultiRobotPuzzle-v2-agents4": 9,
    "MultiRobotPuzzle-v2-agents5": 10, "MultiRobotPuzzleHeavy-v2-agents1": 11, "MultiRobotPuzzleHeavy-v2-agents3": 12,
    "MultiRobotPuzzleHeavy-v2-agents4": 13, "MultiRobotPuzzleHeavy-v2-agents5": 14,
    "MultiRobotPuzzle-v3-agents1": 15, "MultiRobotPuzzle-v3-agents3": 16, "MultiRobotPuzzle-v3-agents4": 17,
    "MultiRobotPuzzle-v3-agents5": 18, "MultiRobotPuzzle-v3-heavy-agents1": 19, "MultiRobotPuzzle-v3-heavy-agents3": 20,
    "MultiRobotPuzzle-v3-heavy-agents4": 21, "MultiRobotPuzzle-v3-heavy-agents5": 22,
}
# env id -> 0 (multi_robot_puzzle_00.py), 2 (multi_robot_puzzle_02.py), 3 (core.py)
ENV_VERSION = {0: 0, 1: 0, 2: 2, 3: 2, 4: 2, 5: 3, 6: 3, **{e: 2 for e in range(7, 15)}, **{e: 3 for e in range(15, 23)}}


def build() -> str:
    """Compile the oracle with its committed Makefile (gcc, -ffp-contract=off)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib(variant: str = "checker"):
    global _lib
    if variant != "checker":
        if variant not in _variants:
            if not os.path.exists(VARIANTS[variant]):
                build()
            _variants[variant] = _bind(ctypes.CDLL(VARIANTS[variant]))
        return _variants[variant]
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = _bind(ctypes.CDLL(_LIB_PATH))
    return _lib


def _bind(L):
    """Declare the argument / return types of the oracle's entry points on a loaded build."""
    c_int, c_float, c_double = ctypes.c_int, ctypes.c_float, ctypes.c_double
    P = ctypes.c_void_p
    for name in ("or_obs_dim", "or_act_dim", "or_n_draws", "or_n_agents", "or_n_blocks", "or_max_episode_steps"):
        getattr(L, name).argtypes = [c_int]
        getattr(L, name).restype = c_int
    L.or_create.argtypes = [c_int]
    L.or_create.restype = P
    L.or_destroy.argtypes = [P]
    L.or_reset.argtypes = [P, P, P, P]
    L.or_step.argtypes = [P, P, P, P, P, P]
    L.or_set_shaped.argtypes = [P, c_double, c_double, c_double]
    L.or_set_frameskip.argtypes = [P, c_int]
    L.or_get_bodies.argtypes = [P, P]
    L.or_get_bodies.restype = c_int
    L.or_get_flags.argtypes = [P, P, P]
    L.or_contact_count.argtypes = [P]
    L.or_contact_count.restype = c_int
    L.or_counters.argtypes = [P, P, P]
    L.or_counters_ex.argtypes = [P, P]
    L.or_proxy_ids.argtypes = [P, P]
    L.or_proxy_ids.restype = c_int
    L.or_sinf.argtypes = [c_float]
    L.or_sinf.restype = c_float
    L.or_cosf.argtypes = [c_float]
    L.or_cosf.restype = c_float
    L.or_sincos_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    L.or_sincos_batch.restype = None
    L.or_rng_u01.argtypes = [ctypes.c_uint64] * 4
    L.or_rng_u01.restype = c_double
    L.or_body_mass.argtypes = [P, c_int, P]
    L.or_body_mass.restype = c_int
    L.or_batch_run.argtypes = [c_int, c_int, c_int, ctypes.c_uint64, ctypes.c_uint64, P, P, c_int, c_int, P, P, P, P]
    L.or_batch_run.restype = ctypes.c_long
    L.or_batch_capacity.argtypes = [c_int, c_int, c_int, ctypes.c_uint64, P, P, c_int, c_int, P]
    L.or_batch_capacity.restype = ctypes.c_long
    L.or_capacity.argtypes = [P, P]
    L.or_work.argtypes = [P, P]
    L.or_batch_work.argtypes = [c_int, c_int, c_int, ctypes.c_uint64, P, P, c_int, c_int, P]
    L.or_batch_work.restype = ctypes.c_long
    L.or_batch_run_window.argtypes = [c_int, c_int, c_int, c_int, ctypes.c_uint64, ctypes.c_uint64, P, P, c_int, c_int,
                                      P, P, P, P]
    L.or_batch_run_window.restype = ctypes.c_long
    L.or_build_kind.argtypes = []
    L.or_build_kind.restype = ctypes.c_char_p
    return L


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


class OracleEnv:
    """One lane of the CPU oracle (one b2World that persists across resets, like the reference)."""

    def __init__(self, env_id: int):
        L = lib()
        self.env_id = env_id
        self.obs_dim = L.or_obs_dim(env_id)
        self.act_dim = L.or_act_dim(env_id)
        self.n_draws = L.or_n_draws(env_id)
        self.n_agents = L.or_n_agents(env_id)
        self.n_blocks = L.or_n_blocks(env_id)
        self.max_episode_steps = L.or_max_episode_steps(env_id)
        self._h = L.or_create(env_id)

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.or_destroy(self._h)
            self._h = None

    def reset(self, draws, action) -> np.ndarray:
        d = np.ascontiguousarray(draws, dtype=np.float64)
        a = np.ascontiguousarray(action, dtype=np.float32)
        assert d.size == self.n_draws and a.size == self.act_dim
        obs = np.zeros(self.obs_dim, np.float64)
        lib().or_reset(self._h, _ptr(d), _ptr(a), _ptr(obs))
        return obs

    def step(self, action):
        a = np.ascontiguousarray(action, dtype=np.float32)
        assert a.size == self.act_dim
        obs = np.zeros(self.obs_dim, np.float64)
        rew = np.zeros(1, np.float64)
        done = np.zeros(1, np.int32)
        kind = np.zeros(1, np.int32)
        lib().or_step(self._h, _ptr(a), _ptr(obs), _ptr(rew), _ptr(done), _ptr(kind))
        return obs, float(rew[0]), bool(done[0]), int(kind[0])

    def set_frameskip(self, frameskip: int):
        lib().or_set_frameskip(self._h, int(frameskip))

    def set_shaped(self, bounds, blk_bounds, puzzle):
        lib().or_set_shaped(self._h, bounds, blk_bounds, puzzle)

    def bodies(self) -> np.ndarray:
        out = np.zeros(6 * (self.n_agents + self.n_blocks), np.float32)
        lib().or_get_bodies(self._h, _ptr(out))
        return out

    def flags(self):
        gc = np.zeros(self.n_agents, np.int32)
        bip = np.zeros(1, np.int32)
        lib().or_get_flags(self._h, _ptr(gc), _ptr(bip))
        return gc, int(bip[0])

    def contact_count(self) -> int:
        return lib().or_contact_count(self._h)

    def counters(self):
        a = np.zeros(1, np.int64)
        b = np.zeros(1, np.int64)
        lib().or_counters(self._h, _ptr(a), _ptr(b))
        return int(a[0]), int(b[0])

    def counters_ex(self) -> dict:
        out = np.zeros(3, np.int64)
        lib().or_counters_ex(self._h, _ptr(out))
        return {"toi_events": int(out[0]), "position_iterations": int(out[1]), "touching_contacts": int(out[2])}

    def body_mass(self, i: int):
        """(mass, inertia about the body origin, local centre x, y) of dynamic body i."""
        out = np.zeros(4, np.float32)
        if lib().or_body_mass(self._h, i, _ptr(out)) != 0:
            raise IndexError(i)
        return tuple(float(v) for v in out)

    def proxy_ids(self) -> np.ndarray:
        out = np.zeros(64, np.int32)
        n = lib().or_proxy_ids(self._h, _ptr(out))
        return out[:n].copy()


def build_kind(variant: str = "checker") -> str:
    return lib(variant).or_build_kind().decode()


def rng_u01(seed: int, lane: int, stream: int, counter: int) -> float:
    return lib().or_rng_u01(seed, lane, stream, counter)


def batch_run(env_id: int, lanes: int, steps: int, seed: int, bounds, threads: int = 1, lane_offset: int = 0,
              outputs: bool = False, max_steps: int = 0, skip: int = 0, variant: str = "checker"):
    """Run `lanes` oracle envs for `skip` + `steps` steps each with the device path's synthetic
    inputs (counter RNG actions and spawns, auto-reset; see or_batch_run) on `threads` OpenMP
    threads; only the last `steps` are timed and counted.  `variant` picks the build (VARIANTS).
    Returns (env_steps, seconds) or, with outputs=True, (env_steps, seconds, bodies, reward_sums,
    episodes)."""
    lo = np.ascontiguousarray([b[0] for b in bounds], dtype=np.float64)
    hi = np.ascontiguousarray([b[1] for b in bounds], dtype=np.float64)
    sec = np.zeros(1, np.float64)
    L = lib(variant)
    nb = 6 * (L.or_n_agents(env_id) + L.or_n_blocks(env_id))
    bodies = np.zeros((lanes, nb), np.float32) if outputs else None
    rsum = np.zeros(lanes, np.float64) if outputs else None
    eps = np.zeros(lanes, np.int32) if outputs else None
    P = lambda a: None if a is None else _ptr(a)  # noqa: E731
    n = L.or_batch_run_window(env_id, lanes, skip, steps, seed, lane_offset, _ptr(lo), _ptr(hi), max_steps, threads,
                              _ptr(sec), P(bodies), P(rsum), P(eps))
    if n < 0:
        raise ValueError("or_batch_run: bad arguments")
    if outputs:
        return int(n), float(sec[0]), bodies, rsum, eps
    return int(n), float(sec[0])


CAPACITY_NAMES = ("contacts", "tree_node_id", "move_buffer", "island_bodies", "island_contacts", "toi_island_bodies",
                  "toi_island_contacts", "tree_node_capacity")


def batch_capacity(env_id: int, lanes: int, steps: int, seed: int, bounds, threads: int = 1, max_steps: int = 0) -> dict:
    """batch_run's workload; returns the per-lane capacity high-water marks (max over lanes)."""
    lo = np.ascontiguousarray([b[0] for b in bounds], dtype=np.float64)
    hi = np.ascontiguousarray([b[1] for b in bounds], dtype=np.float64)
    caps = np.zeros(8, np.int32)
    n = lib().or_batch_capacity(env_id, lanes, steps, seed, _ptr(lo), _ptr(hi), max_steps, threads, _ptr(caps))
    if n < 0:
        raise ValueError("or_batch_capacity: bad arguments")
    return dict(zip(CAPACITY_NAMES, (int(c) for c in caps)))


WORK_NAMES = ("islands", "vel_sweeps", "vel_upd1", "vel_upd2", "vel_levels", "pos_passes", "pos_points",
              "pos_level_points", "toi_vel_upd", "toi_vel_levels", "toi_pos_points", "toi_pos_level_points",
              "sat_calls", "toi_calls", "vel_pipe", "pos_pipe", "isl_units", "isl_concurrent_save", "vel_1wave",
              "vel_2wave")


def batch_work(env_id: int, lanes: int, steps: int, seed: int, bounds, threads: int = 1, max_steps: int = 0) -> np.ndarray:
    """batch_run's workload; returns int64 [steps, lanes, 20]: each launch's work per lane (WORK_NAMES)."""
    lo = np.ascontiguousarray([b[0] for b in bounds], dtype=np.float64)
    hi = np.ascontiguousarray([b[1] for b in bounds], dtype=np.float64)
    out = np.zeros((steps, lanes, len(WORK_NAMES)), np.int64)
    n = lib().or_batch_work(env_id, lanes, steps, seed, _ptr(lo), _ptr(hi), max_steps, threads, _ptr(out))
    if n < 0:
        raise ValueError("or_batch_work: bad arguments")
    return out
