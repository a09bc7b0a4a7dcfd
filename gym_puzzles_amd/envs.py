"""gym-style host classes over the C ABI -- the drop-in surface of gym_puzzles' env classes.

Same class names, constructor arguments, methods, return types and error behaviour as the
reference (``gym_puzzles/envs/__init__.py``):

    MultiRobotPuzzle, MultiRobotPuzzleHeavy          multi_robot_puzzle_00.py:142,606
    MultiRobotPuzzle2, MultiRobotPuzzleHeavy2        multi_robot_puzzle_02.py:126,711
    MultiRobotPuzzleHeavy2ThreeBlock                 build-defined 3-block config
    RobotPuzzleBase                                  core.py:77 (MultiRobotPuzzle-v3; heavy=True too)

Each instance is ONE lane of a device batch (``mrp_ctx`` with n_lanes = 1); the physics runs
on the GPU and the class only moves one row of inputs/outputs.  For thousands of lanes use
``MultiRobotPuzzleVecEnv`` (gym_puzzles_amd/vec_env.py).  Reference behaviours kept:

* the constructor runs ``reset()`` once (multi_robot_puzzle_00.py:209, _02.py:199 via
  ``self.reset()``), drawing from the *global* ``np.random`` (Appendix C.2) and feeding
  ``action_space.sample()`` to the reset step (C.1);
* ``seed(s)`` seeds ``self.np_random`` only (spawns stay on the global RNG) and returns [s];
* ``step`` returns ``(obs float64[O], reward float, done bool, {})``; the TimeLimit is gym's
  wrapper's job (``make()`` adds it), so the kernel's own TimeLimit is off here;
* v2 terminal steps before ``update_params()`` raise ``AttributeError`` (_02.py:554,560,578);
* ``render(mode='rgb_array')`` returns the frame the GPU renderer draws from the lane state
  (uint8 [H, W, 3], ``mrp_render``; scene of multi_robot_puzzle_00.py:528-592 /
  _02.py:590-661); ``mode='human'`` needs a pyglet window, which this build does not open.
"""
from __future__ import annotations

import numpy as np

from ._native import (STATUS_AGENT_OOB, STATUS_BLOCK_OOB, STATUS_FAULT, STATUS_KIND_MASK, STATUS_NONFINITE,
                      STATUS_PUZZLE_COMPLETE, Batch)
from .seeding import make_box, np_random
from .spawn import ENV_VERSION, V2_AGENT_IDS, V3_AGENT_IDS, reference_draws

_DONE_STATUS = {STATUS_PUZZLE_COMPLETE: "puzzle complete!!", STATUS_AGENT_OOB: "agent out of bounds",
                STATUS_BLOCK_OOB: "block out of bounds"}


class _MRPBase:
    metadata = {"render.modes": ["human", "rgb_array", "state_pixels"], "video.frames_per_second": 50}
    env_id = 0
    reward_range = (-float("inf"), float("inf"))
    spec = None

    def __init__(self, device: int = 0):
        self.seed()
        self._b = Batch(self.env_id, 1, device=device)
        self._b.set_time_limit(0)           # gym.wrappers.TimeLimit (make()) owns truncation
        if getattr(self, "frameskip", 1) != 1:   # world.Step calls per step (multi_robot_puzzle_02.py:476-478)
            self._b.set_frameskip(self.frameskip)
        self.num_agents = self._b.n_agents
        self.viewer = None
        self.done_status = None
        self._params_updated = False
        self.set_reward_params()
        low, high = self._obs_bounds()
        self.observation_space = make_box(low, high, dtype=np.float32)
        self.action_space = make_box(-np.ones(self._b.act_dim), np.ones(self._b.act_dim), dtype=np.float32)
        self.reset()

    # -- gym.Env API ---------------------------------------------------------------------
    def seed(self, seed=None):
        self.np_random, seed = np_random(seed)
        return [seed]

    def reset(self):
        draws = reference_draws(self.env_id)          # global np.random, reference order
        act = self.action_space.sample()
        obs = self._b.reset(draws[None], act[None])
        self.done_status = None
        return obs[0].astype(np.float64)

    def step(self, action):
        a = np.asarray(action, dtype=np.float32).reshape(1, -1)
        obs, rew, done, _ = self._b.step(a)
        flags = int(self._b.status[0])
        st = flags & STATUS_KIND_MASK
        self.done_status = _DONE_STATUS.get(st)
        if st != 0 and self._needs_shaped() and not self._params_updated:
            name = "shaped_bounds_penalty" if st == STATUS_AGENT_OOB else (
                "shaped_blk_bounds_penalty" if st == STATUS_BLOCK_OOB else "shaped_puzzle_reward")
            raise AttributeError(f"'{type(self).__name__}' object has no attribute '{name}'")
        # the reference returns {} (multi_robot_puzzle_00.py:521); a broken lane is reported, never
        # raised (SURVEY.md 8b Errors): info['nan'] on a NaN/inf step, info['mrp_fault'] = guard code
        info = {}
        if flags & STATUS_NONFINITE:
            info["nan"] = True
        if flags & STATUS_FAULT:
            info["mrp_fault"] = int(self._b.faults()[0])
        return obs[0].astype(np.float64), float(self._b.reward64[0]), bool(done[0]), info

    def render(self, mode="human", close=False):
        if close:
            return None
        if mode != "rgb_array":
            raise NotImplementedError("only mode='rgb_array' is rendered (no pyglet window in this build)")
        return self._b.render([0])[0]

    def close(self):
        if getattr(self, "_b", None) is not None:
            self._b.close()
            self._b = None

    @property
    def unwrapped(self):
        return self

    # -- tuning hooks ------------------------------------------------------------------------
    def set_reward_params(self, agentDelta=10, agentDistance=None, blockDelta=None, blockDistance=None,
                          puzzleComp=10000, outOfBounds=1000, blkOutOfBounds=100):
        v0 = ENV_VERSION[self.env_id] == 0
        self.weight_deltaAgent = agentDelta
        self.weight_agent_dist = (0.1 if v0 else 0.25) if agentDistance is None else agentDistance
        self.weight_deltaBlock = (50 if v0 else 25) if blockDelta is None else blockDelta
        self.weight_blk_dist = (0.025 if v0 else 0.1) if blockDistance is None else blockDistance
        self.puzzle_complete_reward = puzzleComp
        self.out_of_bounds_penalty = outOfBounds
        self.blk_out_of_bounds_penalty = blkOutOfBounds
        self._b.set_reward_params(self.weight_deltaAgent, self.weight_agent_dist, self.weight_deltaBlock,
                                  self.weight_blk_dist, puzzleComp, outOfBounds, blkOutOfBounds)

    def update_params(self, timestep, decay):
        self._b.update_params(timestep, decay)
        if ENV_VERSION[self.env_id] == 2:
            self.shaped_bounds_penalty = self.out_of_bounds_penalty * decay ** (-timestep)
        self.shaped_blk_bounds_penalty = self.blk_out_of_bounds_penalty * decay ** (-timestep)
        self.shaped_puzzle_reward = self.puzzle_complete_reward * decay ** (-timestep)
        self._params_updated = True

    def update_goal(self, epoch, nb_epochs):
        self._b.update_goal(epoch, nb_epochs)
        self.scaled_epsilon = (25.0 if ENV_VERSION[self.env_id] == 0 else 0.1) * (2 - epoch / nb_epochs)

    def get_deltaAgent(self):
        return self.weight_deltaAgent

    def get_agentDist(self):
        return self.weight_agent_dist

    def get_deltaBlk(self):
        return self.weight_deltaBlock

    def get_blkDist(self):
        return self.weight_blk_dist

    # -- helpers -------------------------------------------------------------------------------
    def _needs_shaped(self):
        return ENV_VERSION[self.env_id] == 2

    def _obs_high(self):
        raise NotImplementedError

    def _obs_bounds(self):
        return -self._obs_high(), self._obs_high()

    @property
    def blks_in_place(self):
        return int(self._b.flags()[0, -1])

    def bodies(self):
        """Dynamic body state (blocks, agents): worldCenter x, y, angle, v x, y, omega."""
        return self._b.bodies()[0].reshape(-1, 6)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class MultiRobotPuzzle(_MRPBase):
    """multi_robot_puzzle_00.py:142 (2 agents, light T block)."""
    env_id = 0
    obs_type = "low-dim"
    heavy = False

    def __init__(self, obs_depth=3, frameskip=4, device: int = 0):
        if self.obs_type != "low-dim":
            raise NotImplementedError("image observations need the renderer (SURVEY.md 8f-3)")
        self._obs_depth = obs_depth
        self.frameskip = 1          # low-dim obs: frameskip 1 (:161-162)
        super().__init__(device)

    def _obs_high(self):
        a = [np.inf] * 4 * self._b.n_agents
        return np.array(a + [np.inf, np.inf, 2 * np.pi, np.inf] + [np.inf] * 16)


class MultiRobotPuzzleHeavy(MultiRobotPuzzle):
    """multi_robot_puzzle_00.py:606 (5 agents, heavy T block)."""
    env_id = 1
    heavy = True


class MultiRobotPuzzle2(_MRPBase):
    """multi_robot_puzzle_02.py:126 (non-holonomic agents with wheels)."""
    env_id = 2
    heavy = False
    unitize = True
    contact_weight = True

    def __init__(self, frameskip=1, num_agents=2, device: int = 0):
        # frameskip (multi_robot_puzzle_02.py:139,146,476-478) is a runtime parameter of the device
        # step; num_agents (:151) sizes the obs / action layout and the per-lane pools, which the
        # device build fixes at compile time: every count from 1 to 5 (Heavy-v0's agent count) has
        # its own env id (include/mrp.h), the T block keeps its single-block layout
        if type(self).env_id in (2, 3):
            key = (int(self.heavy), int(num_agents))
            if key not in V2_AGENT_IDS:
                raise NotImplementedError(f"num_agents={num_agents}: the device build instantiates 1 to 5 agents")
            self.env_id = V2_AGENT_IDS[key]
        elif num_agents != 2:
            raise NotImplementedError("the build-defined 3-block config is instantiated for num_agents=2")
        if int(frameskip) < 1:
            raise ValueError("frameskip must be >= 1")
        self.frameskip = int(frameskip)
        super().__init__(device)

    def _obs_high(self):
        if self._b.n_blocks != 1:           # build-defined layout: unbounded
            return np.full(self._b.obs_dim, np.inf)
        a = [np.inf, np.inf, 2 * np.pi, np.inf, np.inf, np.inf, np.inf, np.inf, np.inf] * self._b.n_agents
        return np.array(a + [np.inf, np.inf, 2 * np.pi, np.inf] + [np.inf] * 16 + [np.inf])


class MultiRobotPuzzleHeavy2(MultiRobotPuzzle2):
    """multi_robot_puzzle_02.py:711 (heavy T block, density 20)."""
    env_id = 3
    heavy = True


class MultiRobotPuzzleHeavy2ThreeBlock(MultiRobotPuzzle2):
    """Build-defined Heavy-v2 3-block square (T + L + I; SURVEY.md 8a-A12, BASELINE configs[4])."""
    env_id = 4
    heavy = True


class RobotPuzzleBase(_MRPBase):
    """core.py:77-418 (MultiRobotPuzzle-v3): holonomic Robots (robot.py:17-73) pushing a T Block
    (blocks.py:17-132) towards a fixed goal; normalised observations.  ``heavy=True`` is the
    reference test's configuration (tests/test_env.py:12): T block at scale 1, density 10.

    Reference quirks kept: the contact detector never sets ``goal_contact`` (core.py:46-61 compares
    Robot wrappers with b2Body objects), so that observation entry and the +0.25 bonus stay 0;
    ``update_params`` / ``update_goal`` store values step() never reads; completion adds
    ``puzzle_complete_reward`` unshaped (core.py:408-410)."""
    env_id = 5

    def __init__(self, num_agents: int = 2, goal_velocity: float = 1.5, block_density: float = 5.0,
                 heavy: bool = False, hardmode: bool = False, device: int = 0):
        # num_agents (core.py:88,106,230) sizes the obs / action layout and the per-lane pools: every
        # count from 1 to 5 has its own env id (include/mrp.h); goal_velocity, block_density and
        # hardmode are stored but never read by the reference (core.py:100-102; heavy picks the block)
        key = (int(bool(heavy)), int(num_agents))
        if key not in V3_AGENT_IDS:
            raise NotImplementedError(f"num_agents={num_agents}: the device build instantiates 1 to 5 agents")
        self.env_id = V3_AGENT_IDS[key]
        self.block_density = block_density
        self.goal_velocity = goal_velocity
        self.heavy = heavy
        self.hardmode = hardmode
        super().__init__(device)

    def set_reward_params(self, agentDelta=10, agentDistance=0.1, blockDelta=50, blockDistance=0.025, puzzleComp=100):
        self.weight_deltaAgent = agentDelta
        self.weight_agent_dist = agentDistance
        self.weight_deltaBlock = blockDelta
        self.weight_blk_dist = blockDistance
        self.puzzle_complete_reward = puzzleComp
        self._b.set_reward_params(agentDelta, agentDistance, blockDelta, blockDistance, puzzleComp)

    def update_params(self, timestep, decay):   # core.py:158-159: stored, never read by step()
        self.shaped_puzzle_reward = self.puzzle_complete_reward * decay ** (-timestep)

    def update_goal(self, epoch, nb_epochs):    # core.py:161-162: stored, never read by step()
        self.scaled_epsilon = 25.0 * (2 - epoch / nb_epochs)

    def _needs_shaped(self):
        return False

    def _return_status(self):
        return self.done_status if self.done_status else "Stayed in bounds"

    def _obs_bounds(self):   # core.py:121-132
        n = self._b.n_agents
        high = [2.5, 2.5, 2 * np.pi, 1.0] * n + [2.5, 2.5, 2 * np.pi] + [1.5] * 16
        low = [-2.5, -2.5, -2 * np.pi, 0.0] * n + [-2.5, -2.5, -2 * np.pi] + [-1.5] * 16
        return np.array(low), np.array(high)

    def _obs_high(self):
        return self._obs_bounds()[1]


ENV_CLASSES = {
    "MultiRobotPuzzle-v0": (MultiRobotPuzzle, 2000),
    "MultiRobotPuzzleHeavy-v0": (MultiRobotPuzzleHeavy, 3000),
    "MultiRobotPuzzle-v2": (MultiRobotPuzzle2, 2000),
    "MultiRobotPuzzleHeavy-v2": (MultiRobotPuzzleHeavy2, 2000),
    "MultiRobotPuzzleHeavy-v2-3block": (MultiRobotPuzzleHeavy2ThreeBlock, 2000),
    "MultiRobotPuzzle-v3": (RobotPuzzleBase, 1500),
}
REWARD_THRESHOLD = {"MultiRobotPuzzle-v3": 110}   # __init__.py:35; the others register 500


class TimeLimit:
    """gym 0.21 ``wrappers.TimeLimit`` (what ``gym.make`` wraps registered envs in)."""

    def __init__(self, env, max_episode_steps):
        self.env = env
        self._max_episode_steps = max_episode_steps
        self._elapsed_steps = None

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return getattr(self.env, name)

    def reset(self, **kw):
        self._elapsed_steps = 0
        return self.env.reset(**kw)

    def step(self, action):
        assert self._elapsed_steps is not None, "Cannot call env.step() before calling reset()"
        obs, reward, done, info = self.env.step(action)
        self._elapsed_steps += 1
        if self._elapsed_steps >= self._max_episode_steps:
            info["TimeLimit.truncated"] = not done
            done = True
        return obs, reward, done, info

    @property
    def unwrapped(self):
        return self.env


def make(env_id: str, **kwargs):
    """``gym.make(id)`` for the registered ids (``gym_puzzles/__init__.py:3-29``)."""
    cls, max_steps = ENV_CLASSES[env_id]
    return TimeLimit(cls(**kwargs), max_steps)


def register_with_gym(alias_suffix: str = "-mi355x") -> dict:
    """Register the reference's ids (gym_puzzles/__init__.py:3-35) with gym's registry when gym is
    importable (it is not in this image), so ``gym.make('MultiRobotPuzzle-v0')`` builds this
    package's class, as the drop-in contract asks.  An id the registry already holds (the
    reference package imported first) is left alone and registered under ``id + alias_suffix``.
    Returns {reference id: registered id}; empty without gym."""
    try:
        from gym.envs.registration import register, registry
    except ImportError:
        return {}
    have = set(getattr(registry, "env_specs", registry).keys()) if hasattr(registry, "keys") or hasattr(registry, "env_specs") else set()
    out = {}
    for name, (cls, max_steps) in ENV_CLASSES.items():
        rid = name if name not in have else name + alias_suffix
        register(id=rid, entry_point=f"gym_puzzles_amd.envs:{cls.__name__}",
                 max_episode_steps=max_steps, reward_threshold=REWARD_THRESHOLD.get(name, 500))
        out[name] = rid
    return out
