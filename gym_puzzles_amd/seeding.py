"""gym 0.21 seeding and ``spaces.Box`` restated in numpy (gym is not importable in this image).

The reference seeds through gym: ``env.seed(s)`` (``multi_robot_puzzle_00.py:211-216``,
``multi_robot_puzzle_02.py:197-201``) and ``env.action_space.seed(s)`` (``train/train.py:65-68``,
``gym_puzzles/tests/test_env.py:17-20``), and every ``reset()`` feeds
``self.action_space.sample()`` to the world (``multi_robot_puzzle_00.py:411``,
``multi_robot_puzzle_02.py:442``).  gym==0.21 (``setup.py:8``) implements these as:

* ``seeding.np_random(seed)``: ``RandomState`` seeded with the little-endian 32-bit words of
  the first 8 bytes of ``sha512(str(seed))`` (``hash_seed``), padded with one zero word
  (``_bigint_from_bytes`` always pads), high zero words dropped (``_int_list_from_bigint``).
* ``Box.sample()`` for a fully bounded float box: ``np_random.uniform(low, high, shape)``
  then ``astype(float32)``.

Only the host-side single-env classes use this; the batched device path uses its counter RNG.
"""
from __future__ import annotations

import hashlib
import os
import struct

import numpy as np


def _bigint_from_bytes(b: bytes) -> int:
    sizeof_int = 4
    padding = sizeof_int - len(b) % sizeof_int
    b += b"\0" * padding
    n = len(b) // sizeof_int
    acc = 0
    for i, v in enumerate(struct.unpack(f"{n}I", b)):
        acc += (2 ** (sizeof_int * 8 * i)) * v
    return acc


def _int_list_from_bigint(x: int):
    if x < 0:
        raise ValueError("seed must be non-negative")
    if x == 0:
        return [0]
    out = []
    while x > 0:
        x, mod = divmod(x, 2 ** 32)
        out.append(mod)
    return out


def create_seed(a=None, max_bytes: int = 8) -> int:
    if a is None:
        return _bigint_from_bytes(os.urandom(max_bytes))
    if isinstance(a, str):
        a = a.encode("utf8")
        a += hashlib.sha512(a).digest()
        return _bigint_from_bytes(a[:max_bytes])
    if isinstance(a, (int, np.integer)):
        return int(a) % 2 ** (8 * max_bytes)
    raise TypeError(f"invalid seed type {type(a)}")


def hash_seed(seed=None, max_bytes: int = 8) -> int:
    if seed is None:
        seed = create_seed(max_bytes=max_bytes)
    h = hashlib.sha512(str(seed).encode("utf8")).digest()
    return _bigint_from_bytes(h[:max_bytes])


def np_random(seed=None):
    """gym.utils.seeding.np_random: (RandomState, seed)."""
    if seed is not None and not (isinstance(seed, (int, np.integer)) and seed >= 0):
        raise ValueError(f"Seed must be a non-negative integer or omitted, not {seed!r}")
    seed = create_seed(seed)
    rng = np.random.RandomState()
    rng.seed(_int_list_from_bigint(hash_seed(seed)))
    return rng, seed


class Box:
    """Bounded float32 ``gym.spaces.Box`` (the only kind the MultiRobotPuzzle envs declare:
    ``multi_robot_puzzle_00.py:202,207``, ``multi_robot_puzzle_02.py:190,195``)."""

    def __init__(self, low, high, shape=None, dtype=np.float32):
        shape = tuple(shape) if shape is not None else np.shape(low)
        self.dtype = np.dtype(dtype)
        self.shape = shape
        self.low = np.full(shape, low, dtype=self.dtype) if np.isscalar(low) else np.asarray(low, self.dtype)
        self.high = np.full(shape, high, dtype=self.dtype) if np.isscalar(high) else np.asarray(high, self.dtype)
        self.bounded_below = -np.inf < self.low
        self.bounded_above = np.inf > self.high
        self.np_random = None
        self.seed()

    def seed(self, seed=None):
        self.np_random, seed = np_random(seed)
        return [seed]

    def sample(self) -> np.ndarray:
        sample = np.empty(self.shape)
        unbounded = ~self.bounded_below & ~self.bounded_above
        upp = ~self.bounded_below & self.bounded_above
        low = ~upp & self.bounded_below & ~self.bounded_above
        bounded = self.bounded_below & self.bounded_above
        sample[unbounded] = self.np_random.normal(size=unbounded[unbounded].shape)
        sample[low] = self.np_random.exponential(size=low[low].shape) + self.low[low]
        sample[upp] = -self.np_random.exponential(size=upp[upp].shape) + self.high[upp]
        sample[bounded] = self.np_random.uniform(low=self.low[bounded], high=self.high[bounded],
                                                 size=bounded[bounded].shape)
        return sample.astype(self.dtype)

    def contains(self, x) -> bool:
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

    def __repr__(self):
        return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"


def make_box(low, high, shape=None, dtype=np.float32):
    """The env's observation/action space: ``gym.spaces.Box`` when gym is importable (SB3's
    wrappers and policies dispatch on ``isinstance(space, gym.spaces.Box)``), else the numpy
    restatement above (same bounds, dtype and sampling algorithm).  stable-baselines3 2.x checks
    for gymnasium spaces, so with SB3 >= 2 installed the space is ``gymnasium.spaces.Box``."""
    try:
        import stable_baselines3
        sb3_major = int(stable_baselines3.__version__.split(".")[0])
    except (ImportError, ValueError, AttributeError):
        sb3_major = 0
    if sb3_major >= 2:
        try:
            from gymnasium import spaces
            return spaces.Box(low, high, shape=shape, dtype=dtype)
        except ImportError:
            pass
    try:
        from gym import spaces
    except ImportError:
        return Box(low, high, shape=shape, dtype=dtype)
    return spaces.Box(low, high, shape=shape, dtype=dtype)
