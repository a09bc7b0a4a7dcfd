"""TEST INFRASTRUCTURE ONLY -- numpy restatement of the stable-baselines3 wrappers the reference
trains with (train/train.py:68 ``Monitor(env)``, train/train.py:80-82 ``VecNormalize(DummyVecEnv)``
with default arguments), the checker of libmrp's on-device statistics (mrp_norm.hip).

stable-baselines3 is not installed here, so this restates its published algorithm (SB3 1.x
``common/running_mean_std.py``, ``common/vec_env/vec_normalize.py``, ``common/monitor.py``):

* ``RunningMeanStd(epsilon=1e-4)``: mean 0, var 1, count 1e-4; ``update(x)`` merges the batch
  moments over axis 0 with Chan et al.'s parallel formula.
* ``VecNormalize(clip_obs=10, clip_reward=10, gamma=0.99, epsilon=1e-8)``: reset updates obs
  statistics and zeroes the discounted returns; step updates obs statistics, normalises obs,
  advances ``returns = returns * gamma + reward``, updates the return statistics, normalises the
  reward with them, normalises done lanes' terminal observations, then ``returns[done] = 0``.
* ``Monitor``: per env, the episode's reward sum (Python floats, in step order) and length.

Batch moments are taken in float64 with two passes, as the device does; SB3's np.mean/np.var of
a float32 batch accumulate in float32, so against SB3 itself this is parity to a tolerance and
otherwise unpinned (no SB3 fixture exists in the reference).
"""
from __future__ import annotations

import numpy as np


class RunningMeanStd:
    def __init__(self, shape=(), epsilon: float = 1e-4):
        self.mean = np.zeros(shape, np.float64)
        self.var = np.ones(shape, np.float64)
        self.count = epsilon

    def update(self, x) -> None:
        x = np.asarray(x, np.float64)
        n = x.shape[0]
        bm = x.sum(axis=0) / n
        bv = ((x - bm) ** 2).sum(axis=0) / n
        delta = bm - self.mean
        tot = self.count + n
        new_mean = self.mean + delta * n / tot
        m2 = self.var * self.count + bv * n + delta * delta * self.count * n / tot
        self.mean, self.var, self.count = new_mean, m2 / tot, tot


class VecNormalizeRef:
    def __init__(self, n_lanes: int, obs_dim: int, clip_obs=10.0, clip_reward=10.0, gamma=0.99, epsilon=1e-8,
                 training: bool = True, norm_obs: bool = True):
        self.norm_obs = norm_obs   # SB3: the observation statistics move only when training and norm_obs
        self.obs_rms = RunningMeanStd((obs_dim,))
        self.ret_rms = RunningMeanStd(())
        self.clip_obs, self.clip_reward, self.gamma, self.epsilon = clip_obs, clip_reward, gamma, epsilon
        self.training = training
        self.returns = np.zeros(n_lanes, np.float64)
        self.ep_ret = np.zeros(n_lanes, np.float64)
        self.ep_len = np.zeros(n_lanes, np.int64)

    def normalize_obs(self, obs):
        x = (np.asarray(obs, np.float64) - self.obs_rms.mean) / np.sqrt(self.obs_rms.var + self.epsilon)
        return np.clip(x, -self.clip_obs, self.clip_obs).astype(np.float32)

    def normalize_reward(self, r):
        x = np.asarray(r, np.float64) / np.sqrt(self.ret_rms.var + self.epsilon)
        return np.clip(x, -self.clip_reward, self.clip_reward).astype(np.float32)

    def reset(self, obs):
        if self.training and self.norm_obs:
            self.obs_rms.update(obs)
        self.returns[:] = 0.0
        self.ep_ret[:] = 0.0
        self.ep_len[:] = 0
        return self.normalize_obs(obs)

    def step(self, obs, reward, done, term_obs=None):
        """Returns (obs', reward', term_obs' for done lanes or None, episode returns, lengths for done lanes)."""
        done = np.asarray(done).astype(bool)
        if self.training and self.norm_obs:
            self.obs_rms.update(obs)
        o = self.normalize_obs(obs)
        if self.training:
            self.returns = self.returns * self.gamma + np.asarray(reward, np.float64)
            self.ret_rms.update(self.returns)
        r = self.normalize_reward(reward)
        t = self.normalize_obs(term_obs) if term_obs is not None else None
        self.ep_ret += np.asarray(reward, np.float64)
        self.ep_len += 1
        er, el = self.ep_ret.copy(), self.ep_len.copy()
        self.ep_ret[done] = 0.0
        self.ep_len[done] = 0
        self.returns[done] = 0.0
        return o, r, t, er, el
