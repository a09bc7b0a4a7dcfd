"""Host-side env classes (gym_puzzles_amd/envs.py, vec_env.py, seeding.py).

CPU: gym 0.21 seeding/Box and TimeLimit logic.  GPU: the single-env classes replay the
reference's own test flow (gym_puzzles/tests/test_env.py) against the committed fixture, and
the SB3-style VecEnv honours SB3's auto-reset contract.
"""
from __future__ import annotations

import os

import numpy as np
import pytest

from gym_puzzles_amd.spawn import reference_draws

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


# ----------------------------------------------------------------------------- CPU
def test_gym_seeding_restatement_properties():
    from gym_puzzles_amd.seeding import Box, _bigint_from_bytes, _int_list_from_bigint, create_seed, np_random
    # _bigint_from_bytes always pads with a zero word (gym 0.21 quirk)
    assert _bigint_from_bytes(b"\x01\x00\x00\x00") == 1
    assert _int_list_from_bigint(2 ** 32 + 5) == [5, 1] and _int_list_from_bigint(0) == [0]
    assert create_seed(17) == 17 and create_seed(2 ** 64 + 3) == 3
    r1, s1 = np_random(17)
    r2, _ = np_random(17)
    assert s1 == 17 and r1.uniform() == r2.uniform()
    with pytest.raises(ValueError):
        np_random(-1)
    sp = Box(-1.0, 1.0, shape=(6,))
    sp.seed(17)
    a = sp.sample()
    assert a.dtype == np.float32 and a.shape == (6,) and np.all(np.abs(a) <= 1) and sp.contains(a)
    sp.seed(17)
    assert np.array_equal(sp.sample(), a)


def test_time_limit_wrapper():
    from gym_puzzles_amd.envs import TimeLimit

    class Fake:
        def reset(self):
            return 0

        def step(self, a):
            return 0, 1.0, a == "end", {}

    env = TimeLimit(Fake(), 3)
    env.reset()
    assert env.step("x")[2] is False and env.step("x")[2] is False
    _, _, done, info = env.step("x")
    assert done and info["TimeLimit.truncated"] is True
    env.reset()
    env.step("x")
    env.step("x")
    _, _, done, info = env.step("end")
    assert done and info["TimeLimit.truncated"] is False


def test_product_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a HIP device is visible")
    from gym_puzzles_amd import MrpError, make
    with pytest.raises(MrpError):
        make("MultiRobotPuzzle-v0")


def test_vec_env_frameskip_only_for_v2():
    """frameskip is a MultiRobotPuzzle2 argument (multi_robot_puzzle_02.py:139,476-478); v0 fixes it to 1
    for low-dim observations (multi_robot_puzzle_00.py:161-162) and RobotPuzzleBase has none, so the
    VecEnv refuses it there before any device work instead of stepping the world k times."""
    from gym_puzzles_amd import MultiRobotPuzzleVecEnv
    for env in ("MultiRobotPuzzle-v0", "MultiRobotPuzzleHeavy-v0", "MultiRobotPuzzle-v3"):
        with pytest.raises(ValueError, match="frameskip"):
            MultiRobotPuzzleVecEnv(env, 4, frameskip=2)
    with pytest.raises(ValueError, match="frameskip"):
        MultiRobotPuzzleVecEnv("MultiRobotPuzzle-v2", 4, frameskip=0)


# ----------------------------------------------------------------------------- GPU
@pytest.mark.gpu
def test_single_env_reference_test_flow(gpu_lib):
    """test_env.py:12-29 flow on gym_puzzles_amd.make('MultiRobotPuzzle-v0'), seed 17."""
    from gym_puzzles_amd import make
    z = np.load(os.path.join(GOLDEN, "scenario_v0_seed17.npz"))
    np.random.seed(0)
    env = make("MultiRobotPuzzle-v0")        # constructor runs reset() once, like the reference
    np.random.seed(17)
    assert env.seed(17) == [17]
    env.action_space.seed(17)
    obs = env.reset()
    assert obs.dtype == np.float64 and obs.shape == env.observation_space.shape == (28,)
    assert np.array_equal(obs.astype(np.float32), z["obs0"])
    for t in range(z["acts"].shape[0]):
        a = env.action_space.sample()
        assert np.array_equal(a, z["acts"][t])
        obs, rew, done, info = env.step(a)
        assert np.array_equal(obs.astype(np.float32), z["obs"][t])
        assert np.float32(rew) == np.float32(z["reward"][t]) and done is False and info == {}
    assert np.array_equal(env.unwrapped.bodies().ravel(), z["bodies"])
    assert env.get_deltaAgent() == 10 and env.get_blkDist() == 0.025
    env.close()


@pytest.mark.gpu
def test_v3_heavy_reference_test_flow(gpu_lib):
    """gym_puzzles/tests/test_env.py itself: make('MultiRobotPuzzle-v3', heavy=True), seed 17,
    obs = reset(), reset(), then action_space.sample() steps until done -- here the 1500-step
    TimeLimit (tests/golden/scenario_v3heavy_seed17.npz)."""
    import random

    from gym_puzzles_amd import make
    z = np.load(os.path.join(GOLDEN, "scenario_v3heavy_seed17.npz"))
    np.random.seed(0)
    env = make("MultiRobotPuzzle-v3", heavy=True)
    assert env.unwrapped.env_id == 6 and env.observation_space.shape == (27,) and env.action_space.shape == (6,)
    assert env.observation_space.high[2] == np.float32(2 * np.pi) and env.observation_space.low[-1] == -1.5
    random.seed(17)
    np.random.seed(17)
    assert env.seed(17) == [17]
    env.action_space.seed(17)
    assert np.array_equal(env.reset().astype(np.float32), z["obs0"][0])
    done = False
    assert np.array_equal(env.reset().astype(np.float32), z["obs0"][1])
    t = 0
    while not done:
        a = env.action_space.sample()
        assert np.array_equal(a, z["acts"][t])
        obs, rew, done, info = env.step(a)
        assert np.array_equal(obs.astype(np.float32), z["obs"][t]), t
        assert rew == pytest.approx(z["reward"][t], rel=1e-12, abs=1e-12) and np.float32(rew) == np.float32(z["reward"][t])
        t += 1
    assert t == z["acts"].shape[0] == 1500 and info == {"TimeLimit.truncated": True}
    assert np.array_equal(env.unwrapped.bodies().ravel(), z["bodies"])
    assert env.get_deltaBlk() == 50 and env.get_agentDist() == 0.1
    env.close()


@pytest.mark.gpu
def test_v3_set_reward_params_and_completion_bonus(gpu_lib, oracle_lib):
    """set_reward_params(puzzleComp=...) is the bonus step() adds (core.py:408-410); a block
    spawned on the goal completes on the reset step and on the first step."""
    from gym_puzzles_amd import Batch
    from oracle import oracle
    b = Batch(5, 2)
    b.set_reward_params(10, 0.1, 50, 0.025, 7.0)
    gx = 5 / 6 * 640 / 30 - 4 / 3 / 30
    draws = np.array([[gx, 8.0, 0.3, 2.0, 2.0, 3.0, 12.0], [10.0, 8.0, 1.0, 2.0, 2.0, 3.0, 12.0]])
    acts = np.zeros((2, 6), np.float32)
    b.reset(draws, acts)
    obs, rew, done, _ = b.step(acts)
    o = [oracle.OracleEnv(5) for _ in range(2)]
    for l in range(2):
        o[l].reset(draws[l], acts[l])
        ob, r, d, k = o[l].step(acts[l])
        assert np.array_equal(obs[l], ob.astype(np.float32)) and int(d) == int(done[l])
    assert done[0] == 1 and done[1] == 0 and b.status[0] == 1
    assert b.reward64[0] > 6.0    # the 7.0 bonus, not the oracle's default 100 nor v0's 10000
    b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name,obs_dim,act_dim", [("MultiRobotPuzzleHeavy-v0", 40, 15), ("MultiRobotPuzzle-v2", 39, 4),
                                                  ("MultiRobotPuzzleHeavy-v2", 39, 4),
                                                  ("MultiRobotPuzzleHeavy-v2-3block", 69, 4),
                                                  ("MultiRobotPuzzle-v3", 27, 6)])
def test_single_env_spaces_and_step(gpu_lib, name, obs_dim, act_dim):
    from gym_puzzles_amd import make
    env = make(name)
    assert env.observation_space.shape == (obs_dim,) and env.action_space.shape == (act_dim,)
    env.update_params(0, 1.0)
    o = env.reset()
    assert o.shape == (obs_dim,)
    for _ in range(20):
        o, r, d, info = env.step(env.action_space.sample())
        assert np.isfinite(o).all() and np.isfinite(r)
    env.close()


def test_num_agents_maps_to_its_env_id():
    """MultiRobotPuzzle2 / MultiRobotPuzzleHeavy2(num_agents=N) (multi_robot_puzzle_02.py:139) for N = 1..5:
    each count has its own env id whose tables hold N agents; other counts raise before any device work."""
    from gym_puzzles_amd import envs
    from gym_puzzles_amd.spawn import ENV_CFG, V2_AGENT_IDS, draw_bounds
    for heavy in (0, 1):
        for n in range(1, 6):
            e = V2_AGENT_IDS[(heavy, n)]
            assert ENV_CFG[e] == (2, n, 1, heavy)
            assert len(draw_bounds(e)) == 1 + 2 * n + 2
    for cls in (envs.MultiRobotPuzzle2, envs.MultiRobotPuzzleHeavy2):
        with pytest.raises(NotImplementedError):
            cls(num_agents=6)
        with pytest.raises(NotImplementedError):
            cls(num_agents=0)
    with pytest.raises(NotImplementedError):
        envs.MultiRobotPuzzleHeavy2ThreeBlock(num_agents=3)
    from gym_puzzles_amd.spawn import V3_AGENT_IDS
    for heavy in (0, 1):
        for n in range(1, 6):
            assert ENV_CFG[V3_AGENT_IDS[(heavy, n)]] == (3, n, 1, heavy)
    with pytest.raises(NotImplementedError):
        envs.RobotPuzzleBase(num_agents=6)


@pytest.mark.gpu
@pytest.mark.parametrize("heavy", [False, True])
@pytest.mark.parametrize("n", [1, 2, 3, 4, 5])
def test_multi_robot_puzzle2_num_agents(gpu_lib, heavy, n):
    """The constructor's spaces follow _02.py:178-194 (9 obs per agent + block 4 + 16 vertices + contact
    weight; 2 action values per agent) and its steps are those of its env id's batch (whose steps
    tests/test_gpu.py compares with the oracle bit for bit): a 1-lane batch given the env's state
    steps to the same obs and rewards."""
    from gym_puzzles_amd import Batch, MultiRobotPuzzle2, MultiRobotPuzzleHeavy2
    env = (MultiRobotPuzzleHeavy2 if heavy else MultiRobotPuzzle2)(num_agents=n)
    assert env.num_agents == n
    assert env.observation_space.shape == (9 * n + 21,) and env.action_space.shape == (2 * n,)
    assert env.observation_space.high[2] == np.float32(2 * np.pi) and env.observation_space.high[9 * n + 2] == np.float32(2 * np.pi)
    env.update_params(0, 1.0)
    mirror = Batch(env.env_id, 1)
    assert mirror.n_agents == n
    mirror.set_time_limit(0)
    mirror.update_params(0, 1.0)
    mirror.set_state(env._b.get_state())
    rs = np.random.RandomState(5 + n)
    for _ in range(40):
        a = rs.uniform(-1, 1, 2 * n).astype(np.float32)
        ob, r, d, _ = env.step(a)
        mo, _, md, _ = mirror.step(a[None])
        assert np.array_equal(ob.astype(np.float32), mo[0]) and r == mirror.reward64[0] and d == bool(md[0])
        if d:
            break
    mirror.close()
    env.close()


@pytest.mark.gpu
@pytest.mark.parametrize("heavy", [False, True])
@pytest.mark.parametrize("n", [1, 3, 5])
def test_robot_puzzle_base_num_agents(gpu_lib, heavy, n):
    """RobotPuzzleBase(num_agents=N, heavy=h): spaces of core.py:121-136 (4 obs per agent in
    [-2.5, 2.5] x2, [-2pi, 2pi], [0, 1]; block 3; 16 vertices in [-1.5, 1.5]; 3 action values per
    agent), steps equal to its env id's batch given the same state."""
    from gym_puzzles_amd import Batch, RobotPuzzleBase
    env = RobotPuzzleBase(num_agents=n, heavy=heavy)
    assert env.num_agents == n and env.observation_space.shape == (4 * n + 19,) and env.action_space.shape == (3 * n,)
    assert env.observation_space.low[3] == 0.0 and env.observation_space.high[4 * n + 2] == np.float32(2 * np.pi)
    mirror = Batch(env.env_id, 1)
    mirror.set_time_limit(0)
    mirror.set_reward_params(10, 0.1, 50, 0.025, 100)
    mirror.set_state(env._b.get_state())
    rs = np.random.RandomState(11 + n)
    for _ in range(40):
        a = rs.uniform(-1, 1, 3 * n).astype(np.float32)
        ob, r, d, _ = env.step(a)
        mo, _, md, _ = mirror.step(a[None])
        assert np.array_equal(ob.astype(np.float32), mo[0]) and r == mirror.reward64[0] and d == bool(md[0])
        if d:
            break
    mirror.close()
    env.close()


@pytest.mark.gpu
def test_vec_env_sb3_contract(gpu_lib):
    from gym_puzzles_amd import Batch, MultiRobotPuzzleVecEnv
    n = 64
    venv = MultiRobotPuzzleVecEnv("MultiRobotPuzzle-v0", n, seed=3, max_episode_steps=25)
    ref = Batch(0, n, seed=3)                  # same RNG keys, no auto-reset
    ref.set_time_limit(25)
    o = venv.reset()
    assert o.shape == (n, 28) and o.dtype == np.float32
    assert np.array_equal(o, ref.reset())
    rs = np.random.RandomState(0)
    seen = 0
    for _ in range(60):
        a = rs.uniform(-1, 1, size=(n, 6)).astype(np.float32)
        obs, rew, done, infos = venv.step(a)
        robs, rrew, rdone, rtrunc = ref.step(a)
        assert np.array_equal(rew, rrew) and np.array_equal(done, rdone.astype(bool))
        for i in np.nonzero(done)[0]:
            seen += 1
            assert np.array_equal(infos[i]["terminal_observation"], robs[i])
            assert infos[i]["TimeLimit.truncated"] == bool(rtrunc[i])
        if done.any():
            robs = ref.reset(mask=done).copy()
        assert np.array_equal(obs, robs)
        assert all("terminal_observation" not in infos[i] for i in np.nonzero(~done)[0])
    assert seen >= n * 2
    assert venv.env_method("update_params", 10, 1.01) == [None] * n
    venv.close()


@pytest.mark.gpu
def test_vec_env_seed_keeps_state_and_rekeys_resets(gpu_lib):
    """seed() re-keys the device RNG for later resets without rebuilding the batch: tuning
    parameters set through env_method survive and step() keeps working (SB3 VecEnv.seed)."""
    from gym_puzzles_amd import MultiRobotPuzzleVecEnv
    n = 32
    a = MultiRobotPuzzleVecEnv("MultiRobotPuzzle-v0", n, seed=3)
    b = MultiRobotPuzzleVecEnv("MultiRobotPuzzle-v0", n, seed=3)
    oa, ob = a.reset(), b.reset()
    assert np.array_equal(oa, ob)
    a.env_method("set_reward_params", 10, 0.1, 50, 0.025)
    assert a.seed(99) == [99 + i for i in range(n)]
    act = np.zeros((n, 6), np.float32)
    ra, rb = a.step(act), b.step(act)            # same lanes, same step: the re-key touches neither
    assert np.array_equal(ra[0], rb[0]) and np.array_equal(ra[1], rb[1])
    a.batch.reset(mask=np.ones(n, np.uint8))
    assert not np.array_equal(a.batch.obs, b.reset())  # later resets draw from the new key
    a.close()
    b.close()


@pytest.mark.gpu
def test_step_torch_rejects_tensors_on_another_device(gpu_lib):
    import torch

    from gym_puzzles_amd import MultiRobotPuzzleVecEnv
    n = 8
    venv = MultiRobotPuzzleVecEnv("MultiRobotPuzzle-v0", n, seed=1)
    venv.reset()
    dev = torch.device("cuda", 0)
    act, obs = torch.zeros((n, 6), device=dev), torch.zeros((n, 28), device=dev)
    rew, done = torch.zeros(n, device=dev), torch.zeros(n, dtype=torch.uint8, device=dev)
    with pytest.raises(ValueError):
        venv.step_torch(act, obs, rew.cpu(), done)
    venv.step_torch(act, obs, rew, done)
    torch.cuda.synchronize(dev)
    assert torch.isfinite(obs).all()
    venv.close()
