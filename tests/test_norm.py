"""On-device VecNormalize + Monitor statistics (mrp_norm.hip) against the numpy
restatement of stable-baselines3's algorithm (oracle/vecnorm_ref.py; SB3 is not installed, so
parity with SB3 itself is unpinned).

Tolerances: batch moments are float64 on both sides but summed in a different order (a
256-thread tree on the device, numpy's pairwise sum here), so statistics agree to rtol 1e-12 and
normalised float32 outputs to 2 ulp-scale (rtol 1e-6, atol 1e-6).  Monitor episode returns are
sequential float64 sums of the same float32 rewards in the same order: bit-exact.
"""
from __future__ import annotations

import os

import numpy as np
import pytest


def test_running_mean_std_merge_is_batch_invariant():
    from oracle.vecnorm_ref import RunningMeanStd
    rs = np.random.RandomState(0)
    x = rs.normal(3.0, 2.0, size=(600, 5))
    a, b = RunningMeanStd((5,)), RunningMeanStd((5,))
    a.update(x)
    for k in range(0, 600, 150):
        b.update(x[k:k + 150])
    np.testing.assert_allclose(a.mean, b.mean, rtol=1e-12)
    np.testing.assert_allclose(a.var, b.var, rtol=1e-9)
    assert a.count == pytest.approx(600 + 1e-4) and b.count == pytest.approx(600 + 1e-4)
    # the epsilon-count prior barely moves the batch moments
    np.testing.assert_allclose(a.mean, x.mean(0), rtol=1e-6)
    np.testing.assert_allclose(a.var, x.var(0), rtol=1e-5)


def test_vecnormalize_restatement_semantics():
    from oracle.vecnorm_ref import VecNormalizeRef
    n = VecNormalizeRef(4, 2, clip_obs=1.0)
    o = n.reset(np.array([[0, 0], [1, 1], [2, 2], [3, 3]], np.float32))
    assert o.dtype == np.float32 and np.all(np.abs(o) <= 1.0)
    r = np.array([1, 2, 3, 4], np.float32)
    _, rn, _, er, el = n.step(np.zeros((4, 2), np.float32), r, np.array([0, 1, 0, 0], np.uint8))
    np.testing.assert_allclose(n.returns, [1, 0, 3, 4])          # returns[done] = 0 after the update
    assert er[1] == 2.0 and el[1] == 1 and n.ep_len[1] == 0 and n.ep_len[0] == 1
    assert np.all(np.abs(rn) <= 10.0)
    n.training = False
    before = n.obs_rms.mean.copy()
    n.step(np.ones((4, 2), np.float32), r, np.zeros(4, np.uint8))
    np.testing.assert_array_equal(n.obs_rms.mean, before)      # frozen statistics in evaluation


@pytest.mark.gpu
def test_device_vecnormalize_matches_restatement(gpu_lib):
    import torch

    from gym_puzzles_amd import Batch, DeviceVecNormalize
    from oracle.vecnorm_ref import VecNormalizeRef
    lanes, steps = 1024, 120
    dev = torch.device("cuda", 0)
    b = Batch(0, lanes, seed=21)
    b.set_auto_reset(True)
    b.set_time_limit(40)                 # every lane finishes episodes inside the run
    O = b.obs_dim
    norm = DeviceVecNormalize(lanes, O, 0)
    ref = VecNormalizeRef(lanes, O)
    obs0 = torch.from_numpy(b.reset().copy()).to(dev)
    nobs = torch.zeros_like(obs0)
    norm.reset(obs0, nobs)
    np.testing.assert_allclose(nobs.cpu().numpy(), ref.reset(obs0.cpu().numpy()), rtol=1e-6, atol=1e-6)
    z = lambda *s, dt=torch.float32: torch.zeros(s, dtype=dt, device=dev)  # noqa: E731
    obs, rew, done, trunc, term = z(lanes, O), z(lanes), z(lanes, dt=torch.uint8), z(lanes, dt=torch.uint8), z(lanes, O)
    nrew, nterm, epr, epl = z(lanes), z(lanes, O), z(lanes, dt=torch.float64), z(lanes, dt=torch.int32)
    s = torch.cuda.current_stream(dev)
    b.set_stream(s.cuda_stream)
    n_done = 0
    for t in range(steps):
        b.step_device(0, obs.data_ptr(), rew.data_ptr(), done.data_ptr(), trunc.data_ptr(), 0, term.data_ptr())
        norm.step(obs, rew, done, nobs, nrew, term, nterm, epr, epl)
        ho, hr, hd, ht = obs.cpu().numpy(), rew.cpu().numpy(), done.cpu().numpy(), term.cpu().numpy()
        o, r, tt, er, el = ref.step(ho, hr, hd, ht)
        np.testing.assert_allclose(nobs.cpu().numpy(), o, rtol=1e-6, atol=1e-6, err_msg=f"obs @{t}")
        np.testing.assert_allclose(nrew.cpu().numpy(), r, rtol=1e-6, atol=1e-6, err_msg=f"reward @{t}")
        m = hd.astype(bool)
        n_done += int(m.sum())
        if m.any():
            np.testing.assert_allclose(nterm.cpu().numpy()[m], tt[m], rtol=1e-6, atol=1e-6, err_msg=f"terminal obs @{t}")
            np.testing.assert_array_equal(epr.cpu().numpy()[m], er[m], err_msg=f"episode return @{t}")
            np.testing.assert_array_equal(epl.cpu().numpy()[m], el[m], err_msg=f"episode length @{t}")
    assert n_done >= 2 * lanes
    st = norm.get_stats()
    np.testing.assert_allclose(st["obs_mean"], ref.obs_rms.mean, rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(st["obs_var"], ref.obs_rms.var, rtol=1e-10)
    np.testing.assert_allclose([st["obs_count"], st["ret_count"]], [ref.obs_rms.count, ref.ret_rms.count], rtol=1e-15)
    np.testing.assert_allclose([st["ret_mean"], st["ret_var"]], [ref.ret_rms.mean, ref.ret_rms.var], rtol=1e-10)
    # evaluation mode freezes the statistics; set/get round-trips them
    norm.training = False
    b.step_device(0, obs.data_ptr(), rew.data_ptr(), done.data_ptr(), trunc.data_ptr(), 0, term.data_ptr())
    norm.step(obs, rew, done, nobs, nrew, term, nterm, epr, epl)
    st2 = norm.get_stats()
    np.testing.assert_array_equal(st2["obs_mean"], st["obs_mean"])
    norm.set_stats(st)
    np.testing.assert_array_equal(norm.get_stats()["obs_var"], st["obs_var"])
    norm.close()
    b.close()


@pytest.mark.gpu
def test_vecnormalize_wrapper_sb3_surface(gpu_lib):
    from gym_puzzles_amd import MultiRobotPuzzleVecEnv, MultiRobotPuzzleVecNormalize
    env = MultiRobotPuzzleVecNormalize(MultiRobotPuzzleVecEnv("MultiRobotPuzzle-v0", 64, seed=5, max_episode_steps=20))
    o = env.reset()
    assert o.shape == (64, 28) and o.dtype == np.float32
    rs = np.random.RandomState(1)
    eps = 0
    for _ in range(45):
        o, r, d, infos = env.step(rs.uniform(-1, 1, size=(64, 6)).astype(np.float32))
        assert np.all(np.abs(o) <= 10.0) and np.all(np.abs(r) <= 10.0)
        for i in np.nonzero(d)[0]:
            eps += 1
            ep = infos[i]["episode"]
            assert 1 <= ep["l"] <= 20 and infos[i]["terminal_observation"].shape == (28,)
    assert eps >= 2 * 64
    env.close()


@pytest.mark.gpu
def test_monitor_sums_the_float64_rewards(gpu_lib):
    """Monitor's episode return sums the env's float64 rewards (SB3's Monitor sums the Python
    floats step() returns), not their float32 roundings: mrp_step_device_ex's reward64 feeds
    mrp_norm_step_device_ex, checked against a sequential float64 sum on the host."""
    import torch

    from gym_puzzles_amd import Batch, DeviceVecNormalize
    lanes, steps = 256, 60
    dev = torch.device("cuda", 0)
    b = Batch(0, lanes, seed=8)
    b.set_auto_reset(True)
    b.set_time_limit(20)
    O = b.obs_dim
    norm = DeviceVecNormalize(lanes, O, 0)
    obs0 = torch.from_numpy(b.reset().copy()).to(dev)
    z = lambda *s, dt=torch.float32: torch.zeros(s, dtype=dt, device=dev)  # noqa: E731
    nobs = torch.zeros_like(obs0)
    norm.reset(obs0, nobs)
    obs, rew, rew64, done = z(lanes, O), z(lanes), z(lanes, dt=torch.float64), z(lanes, dt=torch.uint8)
    nrew, epr, epl = z(lanes), z(lanes, dt=torch.float64), z(lanes, dt=torch.int32)
    b.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    acc = np.zeros(lanes, np.float64)
    n_done = 0
    for _ in range(steps):
        b.step_device(0, obs.data_ptr(), rew.data_ptr(), done.data_ptr(), 0, 0, 0, d_reward64=rew64.data_ptr())
        norm.step(obs, rew, done, nobs, nrew, ep_return=epr, ep_len=epl, reward64=rew64)
        r64, r32, d = rew64.cpu().numpy(), rew.cpu().numpy(), done.cpu().numpy().astype(bool)
        np.testing.assert_array_equal(r64.astype(np.float32), r32)
        acc = acc + r64
        if d.any():
            np.testing.assert_array_equal(epr.cpu().numpy()[d], acc[d])
            acc[d] = 0.0
            n_done += int(d.sum())
    assert n_done >= 2 * lanes
    norm.close()
    b.close()


@pytest.mark.gpu
def test_vecnormalize_save_load_and_eval_flags(gpu_lib, tmp_path):
    """train/test.py:66-68's flow: VecNormalize.load(path, env); env.training = False;
    env.norm_reward = False.  The loaded wrapper carries the saved statistics bit for bit, stops
    updating them once training is off, and returns raw rewards with norm_reward off (raw obs with
    norm_obs off) while the normalised values stay what the statistics give."""
    from gym_puzzles_amd import MultiRobotPuzzleVecEnv, MultiRobotPuzzleVecNormalize
    rs = np.random.RandomState(3)
    act = lambda: rs.uniform(-1, 1, size=(64, 6)).astype(np.float32)  # noqa: E731
    env = MultiRobotPuzzleVecNormalize(MultiRobotPuzzleVecEnv("MultiRobotPuzzle-v0", 64, seed=5, max_episode_steps=20))
    env.reset()
    for _ in range(30):
        env.step(act())
    path = str(tmp_path / "saved_env.pkl")   # train.py:149 / test.py:66 use this exact name
    env.save(path)
    assert os.path.exists(path) and not os.path.exists(path + ".npz")
    st = env.get_stats()
    env.close()

    ev = MultiRobotPuzzleVecNormalize.load(path, MultiRobotPuzzleVecEnv("MultiRobotPuzzle-v0", 64, seed=9,
                                                                        max_episode_steps=20))
    for k, v in st.items():
        np.testing.assert_array_equal(ev.get_stats()[k], v)
    ev.training = False
    ev.norm_reward = False
    ev.reset()
    for _ in range(25):
        o, r, d, infos = ev.step(act())
        np.testing.assert_array_equal(r, ev.get_original_reward())   # raw rewards
        assert np.all(np.abs(o) <= ev.clip_obs)
    for k, v in st.items():   # training off: the statistics did not move
        np.testing.assert_array_equal(ev.get_stats()[k], v)
    ev.norm_obs = False
    o, r, d, infos = ev.step(act())
    np.testing.assert_array_equal(o, ev.get_original_obs())
    ev.close()


def test_restatement_norm_obs_off_freezes_obs_statistics():
    """SB3 VecNormalize updates obs_rms only when training and norm_obs; the returns' statistics
    still move with norm_obs off."""
    from oracle.vecnorm_ref import VecNormalizeRef
    rs = np.random.RandomState(2)
    n = VecNormalizeRef(8, 3, norm_obs=False)
    n.reset(rs.normal(size=(8, 3)))
    for _ in range(5):
        n.step(rs.normal(size=(8, 3)), rs.normal(size=8), np.zeros(8, bool))
    np.testing.assert_array_equal(n.obs_rms.mean, np.zeros(3))
    np.testing.assert_array_equal(n.obs_rms.var, np.ones(3))
    assert n.obs_rms.count == 1e-4 and n.ret_rms.count > 1


@pytest.mark.gpu
def test_device_norm_obs_off_matches_restatement(gpu_lib):
    """norm_obs=False on the device: obs statistics frozen, returns' statistics as SB3's."""
    import torch

    from gym_puzzles_amd import Batch, DeviceVecNormalize
    from oracle.vecnorm_ref import VecNormalizeRef
    lanes, steps = 128, 30
    dev = torch.device("cuda", 0)
    b = Batch(0, lanes, seed=4)
    b.set_auto_reset(True)
    b.set_time_limit(15)
    O = b.obs_dim
    norm = DeviceVecNormalize(lanes, O, 0)
    norm.norm_obs = False
    ref = VecNormalizeRef(lanes, O, norm_obs=False)
    o0 = b.reset().copy()
    nobs = torch.zeros((lanes, O), device=dev)
    norm.reset(torch.from_numpy(o0).to(dev), nobs)
    ref.reset(o0)
    z = lambda *s, dt=torch.float32: torch.zeros(s, dtype=dt, device=dev)  # noqa: E731
    obs, rew, done, nrew = z(lanes, O), z(lanes), z(lanes, dt=torch.uint8), z(lanes)
    b.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    for _ in range(steps):
        b.step_device(0, obs.data_ptr(), rew.data_ptr(), done.data_ptr())
        norm.step(obs, rew, done, nobs, nrew)
        ref.step(obs.cpu().numpy(), rew.cpu().numpy(), done.cpu().numpy())
    st = norm.get_stats()
    np.testing.assert_array_equal(st["obs_mean"], np.zeros(O))
    np.testing.assert_array_equal(st["obs_var"], np.ones(O))
    assert st["obs_count"] == 1e-4
    np.testing.assert_allclose([st["ret_mean"], st["ret_var"], st["ret_count"]],
                               [ref.ret_rms.mean, ref.ret_rms.var, ref.ret_rms.count], rtol=1e-10)
    norm.close()
    b.close()
