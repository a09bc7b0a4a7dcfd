"""ctypes binding of ``libmrp.so`` (the HIP/gfx950 step library; C ABI in ``include/mrp.h``).

The library is built in-tree by ``python -m gym_puzzles_amd.build`` (or
``__graft_entry__.build()``).  There is no CPU fallback: if the shared object is missing
or no HIP device is visible, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from .spawn import ENV_VERSION

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libmrp.so")

MRP_OK = 0
STATUS_RUNNING, STATUS_PUZZLE_COMPLETE, STATUS_AGENT_OOB, STATUS_BLOCK_OOB = 0, 1, 2, 3
STATUS_KIND_MASK, STATUS_NONFINITE, STATUS_FAULT = 0x3F, 0x40, 0x80   # include/mrp.h flag bits
COUNTER_NAMES = ("steps", "resets", "toi_events", "position_iterations", "touching_contacts", "nonfinite_steps",
                 "faulted_lanes")

ENV_IDS = {
    "MultiRobotPuzzle-v0": 0,
    "MultiRobotPuzzleHeavy-v0": 1,
    "MultiRobotPuzzle-v2": 2,
    "MultiRobotPuzzleHeavy-v2": 3,
    "MultiRobotPuzzleHeavy-v2-3block": 4,
    "MultiRobotPuzzle-v3": 5,
    "MultiRobotPuzzle-v3-heavy": 6,      # RobotPuzzleBase(heavy=True) (tests/test_env.py:12)
    # MultiRobotPuzzle2 / MultiRobotPuzzleHeavy2(num_agents=N) (multi_robot_puzzle_02.py:139)
    "MultiRobotPuzzle-v2-agents1": 7, "MultiRobotPuzzle-v2-agents3": 8, "MultiRobotPuzzle-v2-agents4": 9,
    "MultiRobotPuzzle-v2-agents5": 10, "MultiRobotPuzzleHeavy-v2-agents1": 11, "MultiRobotPuzzleHeavy-v2-agents3": 12,
    "MultiRobotPuzzleHeavy-v2-agents4": 13, "MultiRobotPuzzleHeavy-v2-agents5": 14,
    # RobotPuzzleBase(num_agents=N[, heavy=True]) (core.py:86-106)
    "MultiRobotPuzzle-v3-agents1": 15, "MultiRobotPuzzle-v3-agents3": 16, "MultiRobotPuzzle-v3-agents4": 17,
    "MultiRobotPuzzle-v3-agents5": 18, "MultiRobotPuzzle-v3-heavy-agents1": 19, "MultiRobotPuzzle-v3-heavy-agents3": 20,
    "MultiRobotPuzzle-v3-heavy-agents4": 21, "MultiRobotPuzzle-v3-heavy-agents5": 22,
}
MAXF = 24   # csrc/mrp_config.h: fixtures per env (mrp_shapes fills MAXF rows)

# every symbol include/mrp.h declares (tests/test_abi.py checks the .so exports all of them)
EXPORTED = (
    "mrp_env_dims", "mrp_create", "mrp_destroy", "mrp_last_error", "mrp_n_lanes", "mrp_env_id",
    "mrp_set_stream", "mrp_synchronize", "mrp_set_reward_params", "mrp_update_params", "mrp_update_goal",
    "mrp_reset", "mrp_reset_device", "mrp_step", "mrp_step_device", "mrp_step_ex", "mrp_step_device_ex",
    "mrp_step_n_device", "mrp_set_auto_reset", "mrp_set_frameskip", "mrp_set_seed", "mrp_set_schedule", "mrp_get_schedule",
    "mrp_get_bodies", "mrp_get_flags", "mrp_get_faults", "mrp_counters", "mrp_counters_ex", "mrp_state_words", "mrp_get_state", "mrp_set_state",
    "mrp_set_time_limit", "mrp_selftest_sincos", "mrp_debug_stamps", "mrp_debug_stamps_ext",
    "mrp_debug_trace", "mrp_debug_trace_words", "mrp_debug_progress", "mrp_debug_velbench", "mrp_debug_posbench", "mrp_norm_create", "mrp_norm_destroy", "mrp_norm_last_error", "mrp_norm_set_stream",
    "mrp_norm_set_training", "mrp_norm_set_norm_obs", "mrp_norm_reset_device", "mrp_norm_step_device", "mrp_norm_step_device_ex", "mrp_norm_get_stats", "mrp_norm_set_stats",
    "mrp_render", "mrp_render_device", "mrp_get_goals", "mrp_shapes",
)

_lib = None


class MrpError(RuntimeError):
    pass


def load(path: str | None = None) -> ctypes.CDLL:
    """Load libmrp.so (raises if it has not been built: there is no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    LIB_PATH_ = path or os.environ.get("MRP_LIB") or LIB_PATH
    if not os.path.exists(LIB_PATH_):
        raise MrpError(f"{LIB_PATH} not built; run `python -m gym_puzzles_amd.build` (hipcc, gfx950)")
    L = ctypes.CDLL(LIB_PATH_)
    i, d, u64, P = ctypes.c_int, ctypes.c_double, ctypes.c_uint64, ctypes.c_void_p
    ip = ctypes.POINTER(ctypes.c_int)
    L.mrp_env_dims.argtypes = [i, ip, ip, ip, ip, ip, ip]
    L.mrp_create.argtypes = [i, i, i, u64, u64, ctypes.POINTER(P)]
    L.mrp_destroy.argtypes = [P]
    L.mrp_destroy.restype = None
    L.mrp_last_error.argtypes = [P]
    L.mrp_last_error.restype = ctypes.c_char_p
    L.mrp_n_lanes.argtypes = [P]
    L.mrp_env_id.argtypes = [P]
    L.mrp_set_stream.argtypes = [P, P]
    L.mrp_synchronize.argtypes = [P]
    L.mrp_set_reward_params.argtypes = [P, d, d, d, d, d, d, d]
    L.mrp_update_params.argtypes = [P, d, d]
    L.mrp_update_goal.argtypes = [P, d, d]
    L.mrp_reset.argtypes = [P, P, P, P, P]
    L.mrp_reset_device.argtypes = [P, P, P, P, P]
    L.mrp_step.argtypes = [P, P, P, P, P, P, P, P]
    L.mrp_step_device.argtypes = [P, P, P, P, P, P, P, P]
    L.mrp_step_ex.argtypes = [P, P, P, P, P, P, P, P, P]
    L.mrp_step_device_ex.argtypes = [P, P, P, P, P, P, P, P, P]
    L.mrp_step_n_device.argtypes = [P, i, P, P, P, P, P, P, P, P]
    L.mrp_set_seed.argtypes = [P, u64]
    L.mrp_set_schedule.argtypes = [P, i]
    L.mrp_get_schedule.argtypes = [P]
    L.mrp_set_auto_reset.argtypes = [P, i]
    L.mrp_set_frameskip.argtypes = [P, i]
    L.mrp_get_bodies.argtypes = [P, P]
    L.mrp_get_flags.argtypes = [P, P]
    L.mrp_get_faults.argtypes = [P, P]
    L.mrp_counters.argtypes = [P, P, P]
    L.mrp_counters_ex.argtypes = [P, P]
    L.mrp_state_words.argtypes = [i]
    L.mrp_get_state.argtypes = [P, P]
    L.mrp_set_state.argtypes = [P, P]
    L.mrp_set_time_limit.argtypes = [P, i]
    L.mrp_selftest_sincos.argtypes = [i, P, P, P, i]
    L.mrp_render.argtypes = [P, P, i, i, i, P]
    L.mrp_render_device.argtypes = [P, P, i, i, i, P]
    L.mrp_get_goals.argtypes = [P, P]
    L.mrp_shapes.argtypes = [i, P, P, P, P]
    L.mrp_debug_stamps.argtypes = [i, P]
    L.mrp_norm_create.argtypes = [i, i, i, d, d, d, d, ctypes.POINTER(P)]
    L.mrp_norm_destroy.argtypes = [P]
    L.mrp_norm_destroy.restype = None
    L.mrp_norm_last_error.argtypes = [P]
    L.mrp_norm_last_error.restype = ctypes.c_char_p
    L.mrp_norm_set_stream.argtypes = [P, P]
    L.mrp_norm_set_training.argtypes = [P, i]
    L.mrp_norm_set_norm_obs.argtypes = [P, i]
    L.mrp_norm_reset_device.argtypes = [P, P, P]
    L.mrp_norm_step_device.argtypes = [P] * 10
    L.mrp_norm_step_device_ex.argtypes = [P] * 11
    L.mrp_norm_get_stats.argtypes = [P, P]
    L.mrp_norm_set_stats.argtypes = [P, P]
    # every build exports the whole ABI of include/mrp.h (the diagnostics answer MRP_E_STATE outside
    # their -D builds), so an A/B library must be built from this ABI too: a missing symbol raises here
    L.mrp_debug_stamps_ext.argtypes = [i, P, P, P]
    L.mrp_debug_trace.argtypes = [i, P, i]
    L.mrp_debug_trace_words.argtypes = []
    L.mrp_debug_progress.argtypes = [i, ctypes.POINTER(P), i]
    L.mrp_debug_velbench.argtypes = [i, i, i, i, i, P]
    L.mrp_debug_posbench.argtypes = [i, i, i, i, i, P]
    _lib = L
    return L


def trace_words() -> int:
    """Words per lane of mrp_debug_trace's rows (include/mrp.h MRP_TRACE_WORDS): size trace buffers
    from this, never from a literal, so a tool cannot overrun its buffer when the row grows."""
    return int(load().mrp_debug_trace_words())


def env_dims(env_id: int) -> dict:
    L = load()
    vals = [ctypes.c_int() for _ in range(6)]
    rc = L.mrp_env_dims(env_id, *[ctypes.byref(v) for v in vals])
    if rc != MRP_OK:
        raise ValueError(f"unknown env_id {env_id}")
    keys = ("obs_dim", "act_dim", "n_draws", "n_agents", "n_blocks", "max_episode_steps")
    return dict(zip(keys, (v.value for v in vals)))


def shapes(env_id: int) -> dict:
    """Fixture geometry of an env (host-only; creation order, local vertices)."""
    L = load()
    n = ctypes.c_int32()
    fb, cnt = np.zeros(MAXF, np.int32), np.zeros(MAXF, np.int32)
    v = np.zeros((MAXF, 8, 2), np.float32)
    if L.mrp_shapes(env_id, ctypes.byref(n), _p(fb), _p(cnt), _p(v)) != MRP_OK:
        raise ValueError(f"unknown env_id {env_id}")
    return {"n_fix": n.value, "fix_body": fb[:n.value], "counts": cnt[:n.value], "verts": v[:n.value]}


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class Batch:
    """N independent MultiRobotPuzzle worlds on one GPU (one ``mrp_ctx``)."""

    def __init__(self, env_id: int, n_lanes: int, device: int = 0, seed: int = 0, lane_offset: int = 0):
        L = load()
        self.env_id, self.n_lanes, self.device = env_id, n_lanes, device
        self.__dict__.update(env_dims(env_id))
        h = ctypes.c_void_p()
        rc = L.mrp_create(env_id, n_lanes, device, seed, lane_offset, ctypes.byref(h))
        if rc != MRP_OK:
            raise MrpError(f"mrp_create failed ({rc}): {L.mrp_last_error(None).decode()}")
        self._h = h
        self.obs = np.zeros((n_lanes, self.obs_dim), np.float32)
        self.reward = np.zeros(n_lanes, np.float32)
        self.reward64 = np.zeros(n_lanes, np.float64)   # the reference's Python-float rewards
        self.done = np.zeros(n_lanes, np.uint8)
        self.truncated = np.zeros(n_lanes, np.uint8)
        self.status = np.zeros(n_lanes, np.uint8)
        self.terminal_obs = np.zeros((n_lanes, self.obs_dim), np.float32)
        # the output arrays live as long as the batch: their addresses are taken once, so a host step
        # costs one ctypes call (the gym-style single env steps one lane per call)
        self._L = L
        self._out = (self.obs.ctypes.data, self.reward.ctypes.data, self.reward64.ctypes.data, self.done.ctypes.data,
                     self.truncated.ctypes.data, self.status.ctypes.data)
        self._term = self.terminal_obs.ctypes.data

    def _check(self, rc):
        if rc != MRP_OK:
            raise MrpError(load().mrp_last_error(self._h).decode())

    def close(self):
        if getattr(self, "_h", None):
            load().mrp_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def set_reward_params(self, agentDelta=None, agentDistance=None, blockDelta=None, blockDistance=None,
                          puzzleComp=None, outOfBounds=1000, blkOutOfBounds=100):
        v0 = ENV_VERSION[self.env_id] != 2   # v3 defaults equal v0's (core.py:149-155)
        if puzzleComp is None:
            puzzleComp = 100 if ENV_VERSION[self.env_id] == 3 else 10000
        agentDelta = 10 if agentDelta is None else agentDelta
        agentDistance = (0.1 if v0 else 0.25) if agentDistance is None else agentDistance
        blockDelta = (50 if v0 else 25) if blockDelta is None else blockDelta
        blockDistance = (0.025 if v0 else 0.1) if blockDistance is None else blockDistance
        self._check(load().mrp_set_reward_params(self._h, agentDelta, agentDistance, blockDelta, blockDistance,
                                                 puzzleComp, outOfBounds, blkOutOfBounds))

    def update_params(self, timestep, decay):
        self._check(load().mrp_update_params(self._h, float(timestep), float(decay)))

    def update_goal(self, epoch, nb_epochs):
        self._check(load().mrp_update_goal(self._h, float(epoch), float(nb_epochs)))

    def set_frameskip(self, frameskip: int):
        """world.Step calls per env step (MultiRobotPuzzle2(frameskip=k), multi_robot_puzzle_02.py:476-478)."""
        self._check(load().mrp_set_frameskip(self._h, int(frameskip)))

    def set_auto_reset(self, enabled: bool):
        self._check(load().mrp_set_auto_reset(self._h, 1 if enabled else 0))

    def reset(self, draws=None, actions=None, mask=None) -> np.ndarray:
        d = None if draws is None else np.ascontiguousarray(draws, np.float64).reshape(self.n_lanes, self.n_draws)
        a = None if actions is None else np.ascontiguousarray(actions, np.float32).reshape(self.n_lanes, self.act_dim)
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8).reshape(self.n_lanes)
        self._check(load().mrp_reset(self._h, _p(m), _p(d), _p(a), _p(self.obs)))
        return self.obs

    def step(self, actions=None, want_terminal_obs=False):
        if actions is None:
            ap = None
        else:
            a = np.ascontiguousarray(actions, np.float32)
            if a.size != self.n_lanes * self.act_dim:
                raise ValueError(f"actions: expected {self.n_lanes} x {self.act_dim} values, got shape {a.shape}")
            ap = a.ctypes.data
        rc = self._L.mrp_step_ex(self._h, ap, *self._out, self._term if want_terminal_obs else None)
        if rc != MRP_OK:
            self._check(rc)
        return self.obs, self.reward, self.done, self.truncated

    def step_device(self, d_actions, d_obs, d_reward=None, d_done=None, d_trunc=None, d_status=None, d_term=None,
                    d_reward64=None):
        """Asynchronous step on device pointers (ints, e.g. torch ``tensor.data_ptr()``);
        ``d_reward64`` optionally receives the float64 rewards."""
        self._check(load().mrp_step_device_ex(self._h, d_actions, d_obs, d_reward, d_reward64, d_done, d_trunc, d_status,
                                              d_term))

    def step_n_device(self, n_steps, d_actions, d_obs, d_reward=None, d_done=None, d_trunc=None, d_status=None,
                      d_term=None, d_reward64=None):
        """``n_steps`` consecutive steps in one launch (mrp_step_n_device); every array holds
        ``n_steps`` rows of ``n_lanes`` (step-major), device pointers as in step_device."""
        self._check(load().mrp_step_n_device(self._h, int(n_steps), d_actions, d_obs, d_reward, d_reward64, d_done,
                                             d_trunc, d_status, d_term))

    def set_schedule(self, mode):
        """Lane scheduling (mrp_set_schedule): 0 off, 1 costliest-first dispatch, 2 issue priority
        from the previous step's cost, 3 both (True = 1); results are identical in every mode."""
        self._check(load().mrp_set_schedule(self._h, int(mode)))

    def get_schedule(self) -> int:
        """The lane scheduling mode in force (mrp_get_schedule): mrp_create's per-env default until
        set_schedule is called."""
        return int(load().mrp_get_schedule(self._h))

    def set_seed(self, seed: int):
        """Re-key the device RNG (later resets and synthetic actions); lanes, parameters, stream
        and time limit are kept."""
        self._check(load().mrp_set_seed(self._h, int(seed)))

    def set_time_limit(self, max_episode_steps: int):
        self._check(load().mrp_set_time_limit(self._h, int(max_episode_steps)))

    def set_stream(self, stream_ptr):
        self._check(load().mrp_set_stream(self._h, stream_ptr))

    def synchronize(self):
        self._check(load().mrp_synchronize(self._h))

    def bodies(self) -> np.ndarray:
        out = np.zeros((self.n_lanes, 6 * (self.n_agents + self.n_blocks)), np.float32)
        self._check(load().mrp_get_bodies(self._h, _p(out)))
        return out

    def flags(self) -> np.ndarray:
        out = np.zeros((self.n_lanes, self.n_agents + 1), np.int32)
        self._check(load().mrp_get_flags(self._h, _p(out)))
        return out

    def faults(self) -> np.ndarray:
        """Per-lane loop-guard fault codes (0 = none; include/mrp.h mrp_get_faults)."""
        out = np.zeros(self.n_lanes, np.int32)
        self._check(load().mrp_get_faults(self._h, _p(out)))
        return out

    def counters(self):
        a = np.zeros(1, np.int64)
        b = np.zeros(1, np.int64)
        self._check(load().mrp_counters(self._h, _p(a), _p(b)))
        return int(a[0]), int(b[0])

    def counters_ex(self) -> dict:
        """Per-batch counters since creation (mrp_counters_ex; SURVEY.md 5 metrics)."""
        out = np.zeros(8, np.int64)
        self._check(load().mrp_counters_ex(self._h, _p(out)))
        return {k: int(v) for k, v in zip(COUNTER_NAMES, out)}

    def get_state(self) -> np.ndarray:
        w = load().mrp_state_words(self.env_id)
        out = np.zeros((self.n_lanes, w), np.uint32)
        self._check(load().mrp_get_state(self._h, _p(out)))
        return out

    def get_goals(self) -> np.ndarray:
        """block_final_pos per lane: float64 [n_lanes, n_blocks, 3] (v0 px, v2 scaled units)."""
        out = np.zeros((self.n_lanes, self.n_blocks, 3), np.float64)
        self._check(load().mrp_get_goals(self._h, _p(out)))
        return out

    def render(self, lanes=None, width: int | None = None, height: int | None = None) -> np.ndarray:
        """rgb_array frames of the selected lanes: uint8 [n, height, width, 3] (row 0 = top),
        the reference's render(mode='rgb_array') (multi_robot_puzzle_00.py:528-592)."""
        w0, h0 = (1440, 810) if ENV_VERSION[self.env_id] == 2 else (640, 480)   # v0 and v3: 640 x 480
        width, height = width or w0, height or h0
        sel = np.ascontiguousarray(np.arange(self.n_lanes) if lanes is None else np.atleast_1d(lanes), np.int32)
        out = np.zeros((len(sel), height, width, 3), np.uint8)
        self._check(load().mrp_render(self._h, _p(sel), len(sel), width, height, _p(out)))
        return out

    def render_device(self, d_lanes_ptr: int, n: int, width: int, height: int, d_rgb_ptr: int):
        """Asynchronous render into a device buffer (e.g. a torch uint8 tensor's data_ptr())."""
        self._check(load().mrp_render_device(self._h, ctypes.c_void_p(d_lanes_ptr), n, width, height, ctypes.c_void_p(d_rgb_ptr)))

    def set_state(self, state: np.ndarray):
        s = np.ascontiguousarray(state, np.uint32)
        self._check(load().mrp_set_state(self._h, _p(s)))


def selftest_sincos(x: np.ndarray, device: int = 0):
    """Evaluate the device sinf/cosf (glibc-faithful restatement) on ``x``."""
    x = np.ascontiguousarray(x, np.float32)
    s = np.zeros_like(x)
    c = np.zeros_like(x)
    rc = load().mrp_selftest_sincos(device, _p(x), _p(s), _p(c), x.size)
    if rc != MRP_OK:
        raise MrpError(f"mrp_selftest_sincos failed ({rc})")
    return s, c
