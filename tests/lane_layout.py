"""Word offsets of LaneState<ENV> (gym_puzzles_amd/csrc/mrp_world.h), restated for tests that
inject a corrupted lane through mrp_set_state.  tests/test_abi.py checks that the restated size
equals mrp_state_words(env) for every env id, so a layout change that is not mirrored here fails
on the CPU before any GPU test relies on it."""
from __future__ import annotations

# Dims<ENV> (mrp_config.h): NA, NB, NF, CMAX
DIMS = {0: (2, 1, 8, 21), 1: (5, 1, 11, 48), 2: (2, 1, 12, 53), 3: (2, 1, 12, 53), 4: (2, 3, 15, 91),
        5: (2, 1, 8, 21), 6: (2, 1, 8, 21),
        # MultiRobotPuzzle2 / Heavy2 with num_agents = 1, 3, 4, 5 (DimsV2<N>)
        7: (1, 1, 9, 26), 8: (3, 1, 15, 89), 9: (4, 1, 18, 134), 10: (5, 1, 21, 188),
        11: (1, 1, 9, 26), 12: (3, 1, 15, 89), 13: (4, 1, 18, 134), 14: (5, 1, 21, 188),
        # RobotPuzzleBase(num_agents = 1, 3, 4, 5[, heavy=True]) (DimsV3<N>)
        15: (1, 1, 7, 14), 16: (3, 1, 9, 29), 17: (4, 1, 10, 38), 18: (5, 1, 11, 48),
        19: (1, 1, 7, 14), 20: (3, 1, 9, 29), 21: (4, 1, 10, 38), 22: (5, 1, 11, 48)}


def tree_n(nf: int) -> int:
    return 16 if 2 * nf - 1 <= 16 else (32 if 2 * nf - 1 <= 32 else 64)


def move_n(nf: int) -> int:
    return 16 if nf < 16 else 32


def fields(env_id: int):
    """(name, words) in declaration order (32-bit words; doubles / long longs are 2)."""
    na, nb, nf, c = DIMS[env_id]
    nd, tn = na + nb, tree_n(nf)
    f = []
    for n in ("xpx", "xpy", "xs", "xc", "c0x", "c0y", "cx", "cy", "a0", "a", "alpha0", "vx", "vy", "w", "fx", "fy", "tq"):
        f.append((n, nd))
    f.append(("proxy", nf))
    for n in ("tlx", "tly", "thx", "thy", "tpar", "tc1", "tc2", "th", "tud"):
        f.append((n, tn))
    for n in ("root", "freeList", "nodeCount", "moveCount"):
        f.append((n, 1))
    f.append(("moveBuf", move_n(nf)))
    for n in ("cHead", "cFree", "cCount", "cHW"):
        f.append((n, 1))
    for n in ("cnext", "cprev", "cfa", "cfb", "cflags", "ctoiCount", "ctoi", "cfric", "mpc", "mtype",
              "mlnx", "mlny", "mlpx", "mlpy"):
        f.append((n, c))
    for n in ("mpx", "mpy", "mni", "mti", "mid"):
        f.append((n, 2 * c))
    for n in ("inv_dt0", "newFixture", "haveBodies", "episode", "stepCounter", "elapsed", "blks_in_place",
              "prev_blks_in_place"):
        f.append((n, 1))
    f.append(("goal_contact", na))
    f.append(("wall_contact", 1))
    f.append(("fault", 1))
    return f, nd, na, nb


def offsets(env_id: int) -> tuple[dict, int]:
    """{field: word offset} and the total word count (alignment of LaneState as the compiler
    lays it out: doubles on 8 B, the struct padded to 16 B)."""
    f, nd, na, nb = fields(env_id)
    off, w = {}, 0
    for name, n in f:
        off[name] = w
        w += n
    w = (w + 1) // 2 * 2                 # double alignment
    for name, n in (("agent_dist", 2 * na), ("block_distance", 2 * nb), ("goal", 6 * nb), ("toiEvents", 2),
                    ("posIters", 2), ("touching", 2), ("nonfinite", 2)):
        off[name] = w
        w += n
    return off, (w + 3) // 4 * 4         # alignas(16)
