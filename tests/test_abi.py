"""CPU checks of the C-ABI boundary (include/mrp.h <-> gym_puzzles_amd/libmrp.so).

No compute call is made here (no GPU in the CPU suite): the library must load, export every
symbol the header declares, answer the host-only queries, and refuse to create a context
loudly when no HIP device is visible (there is no CPU fallback).
"""
from __future__ import annotations

import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mrp.h")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mrp_[a-z_0-9]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    from gym_puzzles_amd import build as b
    b.build()                       # no-op when up to date
    from gym_puzzles_amd import _native
    return _native.load()


def test_header_declares_the_boundary():
    names = _declared()
    for must in ("mrp_create", "mrp_destroy", "mrp_reset", "mrp_step", "mrp_step_device", "mrp_get_state",
                 "mrp_set_state", "mrp_last_error", "mrp_env_dims", "mrp_counters"):
        assert must in names


def test_library_exports_every_declared_symbol(lib):
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_python_binding_lists_every_symbol(lib):
    from gym_puzzles_amd import _native
    assert sorted(_native.EXPORTED) == _declared()


@pytest.mark.parametrize("env_id,dims", [
    (0, (28, 6, 7, 2, 1, 2000)), (1, (40, 15, 13, 5, 1, 3000)), (2, (39, 4, 7, 2, 1, 2000)),
    (3, (39, 4, 7, 2, 1, 2000)), (4, (69, 4, 9, 2, 3, 2000)), (5, (27, 6, 7, 2, 1, 1500)),
    (6, (27, 6, 7, 2, 1, 1500)),
    # MultiRobotPuzzle2 / Heavy2(num_agents=N): obs 9 N + 21, action 2 N, draws 2 N + 3 (_02.py:178-194)
    (7, (30, 2, 5, 1, 1, 2000)), (8, (48, 6, 9, 3, 1, 2000)), (9, (57, 8, 11, 4, 1, 2000)), (10, (66, 10, 13, 5, 1, 2000)),
    (11, (30, 2, 5, 1, 1, 2000)), (12, (48, 6, 9, 3, 1, 2000)), (13, (57, 8, 11, 4, 1, 2000)), (14, (66, 10, 13, 5, 1, 2000)),
    # RobotPuzzleBase(num_agents=N[, heavy]): obs 4 N + 19, action 3 N, draws 2 N + 3 (core.py:121-136)
    (15, (23, 3, 5, 1, 1, 1500)), (16, (31, 9, 9, 3, 1, 1500)), (17, (35, 12, 11, 4, 1, 1500)), (18, (39, 15, 13, 5, 1, 1500)),
    (19, (23, 3, 5, 1, 1, 1500)), (20, (31, 9, 9, 3, 1, 1500)), (21, (35, 12, 11, 4, 1, 1500)), (22, (39, 15, 13, 5, 1, 1500))])
def test_env_dims(lib, env_id, dims):
    from gym_puzzles_amd import env_dims
    d = env_dims(env_id)
    assert (d["obs_dim"], d["act_dim"], d["n_draws"], d["n_agents"], d["n_blocks"], d["max_episode_steps"]) == dims


def test_env_dims_match_oracle(lib, oracle_lib):
    from gym_puzzles_amd import env_dims
    for e in range(23):
        d = env_dims(e)
        assert d["n_agents"] == oracle_lib.or_n_agents(e) and d["n_blocks"] == oracle_lib.or_n_blocks(e)
        assert d["obs_dim"] == oracle_lib.or_obs_dim(e) and d["act_dim"] == oracle_lib.or_act_dim(e)
        assert d["n_draws"] == oracle_lib.or_n_draws(e)


def test_bad_env_id(lib):
    from gym_puzzles_amd import env_dims
    with pytest.raises(ValueError):
        env_dims(23)
    h = ctypes.c_void_p()
    assert lib.mrp_create(23, 4, 0, 0, 0, ctypes.byref(h)) == -1
    assert b"env_id" in lib.mrp_last_error(None)


def test_state_words_positive(lib):
    w = [lib.mrp_state_words(e) for e in range(23)]
    assert all(x > 0 for x in w) and w[1] > w[0] and w[4] > w[2] and w[5] == w[6] == w[0]
    assert w[7] < w[2] < w[8] < w[9] < w[10] and w[7:11] == w[11:15]
    assert w[15] < w[5] < w[16] < w[17] < w[18] and w[15:19] == w[19:23]
    assert lib.mrp_state_words(23) < 0


def test_no_cpu_fallback_without_device(lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a HIP device is visible")
    from gym_puzzles_amd import Batch, MrpError
    with pytest.raises(MrpError, match="no HIP device"):
        Batch(0, 4)


def test_product_never_imports_the_oracle():
    pkg = os.path.join(ROOT, "gym_puzzles_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".h", ".hip", ".cpp")):
                src = open(os.path.join(dirpath, f)).read()
                assert not re.search(r"^\s*(from|import)\s+oracle", src, flags=re.M), f
                assert "mrp_oracle" not in src and "libmrp_oracle" not in src, f


def test_lane_layout_restatement_matches_library(lib):
    """tests/lane_layout.py (the LaneState word offsets the fault-injection GPU tests write
    through mrp_set_state) sizes every env's lane exactly as the library does."""
    from lane_layout import offsets
    for e in range(23):
        off, words = offsets(e)
        assert words == lib.mrp_state_words(e), e
        assert off["nonfinite"] + 2 <= words and off["fault"] < off["agent_dist"]


def test_status_flag_bits_agree():
    src = open(HEADER).read()
    from gym_puzzles_amd import _native
    assert f"#define MRP_STATUS_NONFINITE 0x{_native.STATUS_NONFINITE:x}" in src
    assert f"#define MRP_STATUS_FAULT 0x{_native.STATUS_FAULT:x}" in src
    assert f"#define MRP_STATUS_KIND_MASK 0x{_native.STATUS_KIND_MASK:x}" in src
