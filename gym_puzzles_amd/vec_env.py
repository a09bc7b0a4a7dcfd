"""SB3-style vectorised env over one device batch (reference callers
``train/train.py:63-82`` build ``DummyVecEnv([make_env] * n_envs)`` + ``VecNormalize``).

``MultiRobotPuzzleVecEnv(env_id, num_envs)`` exposes the stable-baselines3 ``VecEnv``
interface (reset / step_async / step_wait / step / close / seed / get_attr / set_attr /
env_method / env_is_wrapped) with SB3's auto-reset semantics: a finished lane is reset inside
the same ``mrp_step`` call on the GPU, ``obs`` holds its new first observation and
``infos[i]["terminal_observation"]`` the last one; ``infos[i]["TimeLimit.truncated"]`` marks
TimeLimit ends.  Spawns and reset actions then come from the device counter RNG (keyed by
seed and global lane), not from ``np.random``.

``step_torch`` is the zero-copy variant for a policy that lives on the same GPU: actions and
outputs are torch CUDA tensors and nothing crosses PCIe.
"""
from __future__ import annotations

import numpy as np

from ._native import Batch, env_dims
from .seeding import Box

_ID = {"MultiRobotPuzzle-v0": 0, "MultiRobotPuzzleHeavy-v0": 1, "MultiRobotPuzzle-v2": 2,
       "MultiRobotPuzzleHeavy-v2": 3, "MultiRobotPuzzleHeavy-v2-3block": 4}


class MultiRobotPuzzleVecEnv:
    def __init__(self, env_id, num_envs: int, device: int = 0, seed: int = 0, lane_offset: int = 0,
                 max_episode_steps: int | None = None):
        self.env_index = _ID[env_id] if isinstance(env_id, str) else int(env_id)
        d = env_dims(self.env_index)
        self.num_envs = num_envs
        self.device = device
        self._seed = seed
        self._lane_offset = lane_offset
        self.observation_space = Box(-np.inf, np.inf, shape=(d["obs_dim"],), dtype=np.float32)
        self.action_space = Box(-1.0, 1.0, shape=(d["act_dim"],), dtype=np.float32)
        self.max_episode_steps = d["max_episode_steps"] if max_episode_steps is None else max_episode_steps
        self._b = None
        self._make_batch()
        self._actions = None
        self._attrs = {}

    def _make_batch(self):
        if self._b is not None:
            self._b.close()
        self._b = Batch(self.env_index, self.num_envs, device=self.device, seed=self._seed,
                        lane_offset=self._lane_offset)
        self._b.set_time_limit(self.max_episode_steps)
        self._b.set_auto_reset(True)

    # -- VecEnv API ------------------------------------------------------------------------
    def reset(self) -> np.ndarray:
        return self._b.reset().copy()

    def step_async(self, actions) -> None:
        self._actions = np.ascontiguousarray(actions, dtype=np.float32).reshape(self.num_envs, -1)

    def step_wait(self):
        obs, rew, done, trunc = self._b.step(self._actions, want_terminal_obs=True)
        infos = [{} for _ in range(self.num_envs)]
        for i in np.nonzero(done)[0]:
            infos[i]["terminal_observation"] = self._b.terminal_obs[i].copy()
            infos[i]["TimeLimit.truncated"] = bool(trunc[i])
        return obs.copy(), rew.copy(), done.astype(bool), infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def close(self) -> None:
        if self._b is not None:
            self._b.close()
            self._b = None

    def seed(self, seed=None):
        """Re-key the device RNG (takes effect from the next reset); returns one seed per env."""
        self._seed = 0 if seed is None else int(seed)
        self._make_batch()
        return [self._seed + i for i in range(self.num_envs)]

    def get_attr(self, attr_name, indices=None):
        idx = self._indices(indices)
        if attr_name in ("observation_space", "action_space", "max_episode_steps"):
            return [getattr(self, attr_name)] * len(idx)
        if attr_name not in self._attrs:
            raise AttributeError(attr_name)
        return [self._attrs[attr_name]] * len(idx)

    def set_attr(self, attr_name, value, indices=None):
        self._attrs[attr_name] = value

    def env_method(self, method_name, *args, indices=None, **kwargs):
        """Tuning hooks apply to every lane of the batch (one parameter block per ctx)."""
        if method_name not in ("set_reward_params", "update_params", "update_goal"):
            raise AttributeError(method_name)
        getattr(self._b, method_name)(*args, **kwargs)
        return [None] * len(self._indices(indices))

    def env_is_wrapped(self, wrapper_class, indices=None):
        return [False] * len(self._indices(indices))

    def get_images(self):
        raise NotImplementedError("rendering is not built yet (SURVEY.md 8f-3)")

    def _indices(self, indices):
        if indices is None:
            return list(range(self.num_envs))
        if isinstance(indices, int):
            return [indices]
        return list(indices)

    # -- zero-copy device path -----------------------------------------------------------------
    def step_torch(self, actions, obs, reward, done, truncated=None, terminal_obs=None):
        """One step on torch CUDA tensors (float32 [N, A] actions, [N, O] obs, [N] reward,
        uint8 [N] done/truncated, optional [N, O] terminal_obs), asynchronous on the current
        torch stream."""
        import torch
        self._b.set_stream(torch.cuda.current_stream().cuda_stream)
        ptr = (lambda t: 0 if t is None else t.data_ptr())
        self._b.step_device(ptr(actions), obs.data_ptr(), reward.data_ptr(), done.data_ptr(), ptr(truncated), 0,
                            ptr(terminal_obs))

    @property
    def batch(self) -> Batch:
        return self._b
