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

When stable-baselines3 is importable the class derives from its ``VecEnv`` and the spaces are
``gym.spaces.Box`` (what SB3's wrappers check with ``isinstance``); neither package is in this
image, so that path is untested here (parity unpinned) and ``MultiRobotPuzzleVecNormalize`` is
the tested way to get VecNormalize + Monitor.
"""
from __future__ import annotations

import numpy as np

from ._native import ENV_IDS, STATUS_FAULT, STATUS_NONFINITE, Batch, env_dims
from .spawn import ENV_CFG, V2_AGENT_IDS, V3_AGENT_IDS
from .seeding import make_box

try:   # SB3 1.x/2.x: VecEnv(num_envs, observation_space, action_space)
    from stable_baselines3.common.vec_env.base_vec_env import VecEnv as _VecEnvBase
except ImportError:
    _VecEnvBase = object

_ID = dict(ENV_IDS)


def _lane_flags(batch: Batch, status: np.ndarray, infos: list) -> None:
    """Per-lane failure report (SURVEY.md 8b Errors): ``info['nan']`` for a lane whose step
    produced a NaN / inf, ``info['mrp_fault']`` = the loop-guard code of a lane whose guard has
    tripped (include/mrp.h status flag bits).  Never raises; healthy lanes get no extra keys."""
    nan = np.nonzero(status & STATUS_NONFINITE)[0]
    for i in nan:
        infos[i]["nan"] = True
    bad = np.nonzero(status & STATUS_FAULT)[0]
    if bad.size:
        codes = batch.faults()
        for i in bad:
            infos[i]["mrp_fault"] = int(codes[i])


class MultiRobotPuzzleVecEnv(_VecEnvBase):
    def __init__(self, env_id, num_envs: int, device: int = 0, seed: int = 0, lane_offset: int = 0,
                 max_episode_steps: int | None = None, frameskip: int = 1, num_agents: int | None = None):
        self.env_index = _ID[env_id] if isinstance(env_id, str) else int(env_id)
        if num_agents is not None and num_agents != env_dims(self.env_index)["n_agents"]:
            # MultiRobotPuzzle2 / Heavy2(num_agents=N) (multi_robot_puzzle_02.py:139): the env id of that count
            cfg = ENV_CFG[self.env_index]
            key = (cfg[3], int(num_agents))
            ids = V2_AGENT_IDS if cfg[0] == 2 and cfg[2] == 1 else (V3_AGENT_IDS if cfg[0] == 3 else {})
            if key not in ids:
                raise NotImplementedError(f"num_agents={num_agents} is not instantiated for env {env_id!r}")
            self.env_index = ids[key]
        d = env_dims(self.env_index)
        self.num_envs = num_envs
        self.device = device
        self._seed = seed
        self._lane_offset = lane_offset
        # MultiRobotPuzzle2(frameskip=k) (multi_robot_puzzle_02.py:139,476-478): world.Step calls per env
        # step.  Only the v2 classes take it: v0 fixes frameskip 1 for its low-dim observations
        # (multi_robot_puzzle_00.py:161-162) and RobotPuzzleBase has none (core.py:77-418)
        self.frameskip = int(frameskip)
        if self.frameskip < 1:
            raise ValueError("frameskip must be >= 1")
        if self.frameskip != 1 and ENV_CFG[self.env_index][0] != 2:
            raise ValueError(f"frameskip={frameskip}: only the MultiRobotPuzzle2 envs (v2) repeat world.Step per env step")
        self.observation_space = make_box(-np.inf, np.inf, shape=(d["obs_dim"],), dtype=np.float32)
        self.action_space = make_box(-1.0, 1.0, shape=(d["act_dim"],), dtype=np.float32)
        self.max_episode_steps = d["max_episode_steps"] if max_episode_steps is None else max_episode_steps
        # everything get_attr / step need exists before SB3's base __init__ runs (SB3 2.x queries
        # get_attr("render_mode") from it)
        self._attrs = {"render_mode": None}
        self._actions = None
        self._b = None
        self._make_batch()
        if _VecEnvBase is not object:
            _VecEnvBase.__init__(self, num_envs, self.observation_space, self.action_space)

    def _make_batch(self):
        if self._b is not None:
            self._b.close()
        self._b = Batch(self.env_index, self.num_envs, device=self.device, seed=self._seed,
                        lane_offset=self._lane_offset)
        self._b.set_time_limit(self.max_episode_steps)
        self._b.set_auto_reset(True)
        if self.frameskip != 1:
            self._b.set_frameskip(self.frameskip)

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
        _lane_flags(self._b, self._b.status, infos)
        return obs.copy(), rew.copy(), done.astype(bool), infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def close(self) -> None:
        if self._b is not None:
            self._b.close()
            self._b = None

    def seed(self, seed=None):
        """Re-key the device RNG (takes effect from the next reset, as SB3's VecEnv.seed does);
        lane state, tuning parameters, stream and time limit are kept.  Returns one seed per env."""
        self._seed = 0 if seed is None else int(seed)
        self._b.set_seed(self._seed)
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
        """One rgb_array frame per env (SB3 VecEnv.get_images; frames from mrp_render)."""
        return list(self._b.render())

    def _indices(self, indices):
        if indices is None:
            return list(range(self.num_envs))
        if isinstance(indices, int):
            return [indices]
        return list(indices)

    # -- zero-copy device path -----------------------------------------------------------------
    def step_torch(self, actions, obs, reward, done, truncated=None, terminal_obs=None, reward64=None, status=None):
        """One step on torch CUDA tensors on this env's device (float32 [N, A] actions, [N, O] obs,
        [N] reward, uint8 [N] done/truncated/status, optional [N, O] terminal_obs and float64 [N]
        reward64), asynchronous on that device's current torch stream."""
        import torch
        dev = torch.device("cuda", self.device)
        for name, t in (("actions", actions), ("obs", obs), ("reward", reward), ("done", done), ("truncated", truncated),
                        ("terminal_obs", terminal_obs), ("reward64", reward64), ("status", status)):
            if t is not None and t.device != dev:
                raise ValueError(f"step_torch: {name} is on {t.device}, this VecEnv runs on {dev}")
        self._b.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        ptr = (lambda t: 0 if t is None else t.data_ptr())
        self._b.step_device(ptr(actions), obs.data_ptr(), reward.data_ptr(), done.data_ptr(), ptr(truncated), ptr(status),
                            ptr(terminal_obs), ptr(reward64))

    @property
    def batch(self) -> Batch:
        return self._b


class DeviceVecNormalize:
    """stable-baselines3 ``VecNormalize`` + ``Monitor`` statistics kept on the GPU (libmrp's
    ``mrp_norm_*``).  The reference wraps every env in ``Monitor`` and the vector
    env in ``VecNormalize`` with default arguments (``train/train.py:68,80-82``).  All arrays are
    torch CUDA tensors on ``device``; calls are asynchronous on the current torch stream."""

    def __init__(self, n_lanes: int, obs_dim: int, device: int = 0, clip_obs: float = 10.0, clip_reward: float = 10.0,
                 gamma: float = 0.99, epsilon: float = 1e-8):
        import ctypes

        from ._native import MrpError, load
        self._L, self._err = load(), MrpError
        self.n_lanes, self.obs_dim, self.device = n_lanes, obs_dim, device
        h = ctypes.c_void_p()
        rc = self._L.mrp_norm_create(n_lanes, obs_dim, device, clip_obs, clip_reward, gamma, epsilon, ctypes.byref(h))
        if rc != 0:
            raise MrpError(f"mrp_norm_create failed ({rc}): {self._L.mrp_norm_last_error(None).decode()}")
        self._h = h
        self._training = True
        self._norm_obs = True

    def _check(self, rc):
        if rc != 0:
            raise self._err(self._L.mrp_norm_last_error(self._h).decode())

    def _sync_stream(self):
        import torch
        self._check(self._L.mrp_norm_set_stream(self._h, torch.cuda.current_stream(self.device).cuda_stream))

    @property
    def training(self) -> bool:
        return self._training

    @training.setter
    def training(self, value: bool):
        self._training = bool(value)
        self._check(self._L.mrp_norm_set_training(self._h, int(self._training)))

    @property
    def norm_obs(self) -> bool:
        return self._norm_obs

    @norm_obs.setter
    def norm_obs(self, value: bool):
        """SB3 VecNormalize.norm_obs: the observation statistics only move while it is set."""
        self._norm_obs = bool(value)
        self._check(self._L.mrp_norm_set_norm_obs(self._h, int(self._norm_obs)))

    def reset(self, obs, obs_out):
        self._sync_stream()
        self._check(self._L.mrp_norm_reset_device(self._h, obs.data_ptr(), obs_out.data_ptr()))

    def step(self, obs, reward, done, obs_out, reward_out, term_obs=None, term_out=None, ep_return=None, ep_len=None,
             reward64=None):
        """``reward64`` (float64 [N], optional): the env's float64 rewards, which Monitor's
        episode return then sums (SB3's Monitor sums the env's Python-float rewards)."""
        ptr = (lambda t: None if t is None else t.data_ptr())
        self._sync_stream()
        self._check(self._L.mrp_norm_step_device_ex(self._h, ptr(obs), ptr(reward), ptr(reward64), ptr(done), ptr(term_obs),
                                                     ptr(obs_out), ptr(reward_out), ptr(term_out), ptr(ep_return), ptr(ep_len)))

    def get_stats(self) -> dict:
        st = np.zeros(2 * self.obs_dim + 4, np.float64)
        self._check(self._L.mrp_norm_get_stats(self._h, st.ctypes.data))
        D = self.obs_dim
        return {"obs_mean": st[:D], "obs_var": st[D:2 * D], "obs_count": st[2 * D], "ret_mean": st[2 * D + 1],
                "ret_var": st[2 * D + 2], "ret_count": st[2 * D + 3]}

    def set_stats(self, stats: dict) -> None:
        st = np.concatenate([np.asarray(stats["obs_mean"], np.float64), np.asarray(stats["obs_var"], np.float64),
                             [stats["obs_count"], stats["ret_mean"], stats["ret_var"], stats["ret_count"]]])
        self._check(self._L.mrp_norm_set_stats(self._h, np.ascontiguousarray(st).ctypes.data))

    def close(self):
        if getattr(self, "_h", None):
            self._L.mrp_norm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class MultiRobotPuzzleVecNormalize:
    """``VecNormalize(MultiRobotPuzzleVecEnv)`` with ``Monitor`` episode records, computed on the
    device.  Same VecEnv surface as SB3's wrapper: ``reset()`` / ``step(actions)`` return host
    numpy arrays (normalised obs and reward), ``infos[i]`` carry ``terminal_observation``
    (normalised), ``TimeLimit.truncated`` and Monitor's ``episode`` = {"r", "l"} for finished
    lanes; ``get_original_obs()`` / ``get_original_reward()`` give the raw values."""

    def __init__(self, venv: MultiRobotPuzzleVecEnv, training: bool = True, norm_obs: bool = True, norm_reward: bool = True,
                 clip_obs: float = 10.0, clip_reward: float = 10.0, gamma: float = 0.99, epsilon: float = 1e-8):
        import torch
        self.venv = venv
        # SB3 semantics: the flags choose what step()/reset() return; while `training` is set the
        # returns' statistics are updated, and the observation statistics only when norm_obs is set
        self.norm_reward = bool(norm_reward)
        self.clip_obs, self.clip_reward, self.gamma, self.epsilon = clip_obs, clip_reward, gamma, epsilon
        self.num_envs, self.observation_space, self.action_space = venv.num_envs, venv.observation_space, venv.action_space
        N, O = venv.num_envs, venv.observation_space.shape[0]
        dev = torch.device("cuda", venv.device)
        self.norm = DeviceVecNormalize(N, O, venv.device, clip_obs, clip_reward, gamma, epsilon)
        self.norm.training = training
        self.norm.norm_obs = norm_obs
        z = lambda *s, dt=torch.float32: torch.zeros(s, dtype=dt, device=dev)  # noqa: E731
        self._act, self._obs, self._rew = z(N, venv.action_space.shape[0]), z(N, O), z(N)
        self._done, self._trunc, self._term = z(N, dt=torch.uint8), z(N, dt=torch.uint8), z(N, O)
        self._nobs, self._nrew, self._nterm = z(N, O), z(N), z(N, O)
        self._epr, self._epl = z(N, dt=torch.float64), z(N, dt=torch.int32)
        self._rew64 = z(N, dt=torch.float64)
        self._status = z(N, dt=torch.uint8)

    @property
    def training(self):
        return self.norm.training

    @training.setter
    def training(self, v):
        self.norm.training = v

    @property
    def norm_obs(self):
        return self.norm.norm_obs

    @norm_obs.setter
    def norm_obs(self, v):
        self.norm.norm_obs = v

    def reset(self):
        import torch
        self._obs.copy_(torch.from_numpy(self.venv.reset()))
        self.norm.reset(self._obs, self._nobs)
        return (self._nobs if self.norm_obs else self._obs).cpu().numpy()

    def step(self, actions):
        import torch
        self._act.copy_(torch.as_tensor(np.asarray(actions, np.float32).reshape(self.num_envs, -1)))
        self.venv.step_torch(self._act, self._obs, self._rew, self._done, self._trunc, self._term, self._rew64, self._status)
        self.norm.step(self._obs, self._rew, self._done, self._nobs, self._nrew, self._term, self._nterm, self._epr, self._epl,
                       self._rew64)
        obs = (self._nobs if self.norm_obs else self._obs).cpu().numpy()
        rew = (self._nrew if self.norm_reward else self._rew).cpu().numpy()
        done, trunc = self._done.cpu().numpy().astype(bool), self._trunc.cpu().numpy().astype(bool)
        infos = [{} for _ in range(self.num_envs)]
        idx = np.nonzero(done)[0]
        if idx.size:
            term = (self._nterm if self.norm_obs else self._term).cpu().numpy()
            epr, epl = self._epr.cpu().numpy(), self._epl.cpu().numpy()
            for i in idx:
                infos[i]["terminal_observation"] = term[i].copy()
                infos[i]["TimeLimit.truncated"] = bool(trunc[i])
                infos[i]["episode"] = {"r": round(float(epr[i]), 6), "l": int(epl[i])}
        _lane_flags(self.venv.batch, self._status.cpu().numpy(), infos)
        return obs, rew, done, infos

    def get_original_obs(self):
        return self._obs.cpu().numpy()

    # ---- persistence (SB3's VecNormalize.save / VecNormalize.load, train/test.py:66) --------
    # SB3 pickles the wrapper; this build stores the same statistics and settings in an .npz
    # (nothing in the file is executed on load).
    def save(self, save_path: str) -> None:
        """Writes exactly `save_path` (train.py:149 saves to 'models/<run>/saved_env.pkl' and
        test.py:66 loads that same path back; np.savez on a bare path would append '.npz')."""
        st = self.norm.get_stats()
        with open(save_path, "wb") as f:
            np.savez(f, **st, clip_obs=self.clip_obs, clip_reward=self.clip_reward, gamma=self.gamma,
                     epsilon=self.epsilon, training=self.training, norm_obs=self.norm_obs, norm_reward=self.norm_reward)

    @classmethod
    def load(cls, load_path: str, venv: MultiRobotPuzzleVecEnv) -> "MultiRobotPuzzleVecNormalize":
        with np.load(load_path, allow_pickle=False) as z:
            d = {k: z[k] for k in z.files}
        self = cls(venv, training=bool(d["training"]), norm_obs=bool(d["norm_obs"]), norm_reward=bool(d["norm_reward"]),
                   clip_obs=float(d["clip_obs"]), clip_reward=float(d["clip_reward"]), gamma=float(d["gamma"]),
                   epsilon=float(d["epsilon"]))
        self.norm.set_stats({k: d[k] for k in ("obs_mean", "obs_var", "obs_count", "ret_mean", "ret_var", "ret_count")})
        return self

    def get_stats(self) -> dict:
        return self.norm.get_stats()

    def get_original_reward(self):
        return self._rew.cpu().numpy()

    def get_images(self):   # VecEnvWrapper passes rendering through (VecVideoRecorder, test.py:61-63)
        return self.venv.get_images()

    def env_method(self, method_name, *args, indices=None, **kwargs):
        return self.venv.env_method(method_name, *args, indices=indices, **kwargs)

    def get_attr(self, attr_name, indices=None):
        return self.venv.get_attr(attr_name, indices)

    def close(self):
        self.norm.close()
        self.venv.close()
