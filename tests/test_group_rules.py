"""Host restatements of two round-4 exactness arguments (CPU only; the device code itself is
covered bit for bit against the oracle by tests/test_gpu.py).

1. The grouped SAT edge scan (mrp_world.h find_max_separation_grp): G lanes each scan edges
   sub, sub + G, ... with the reference's strict-greater rule, then reduce pairwise (larger
   separation, smaller edge among equals; an edge that never beat -FLT_MAX or is NaN takes no
   part).  Must give the reference's sequential b2FindMaxSeparation result for any values.
2. The sparse early-exit schedule (mrp_world.h exit_mask / Snap::step, sweep_pairs, lanes_sweeps):
   every compare point k has a snapshot from exactly two sweeps before and iters - k even, so a
   repeat found there gives the state after all `iters` sweeps.
"""
import itertools
import math
import random
import struct

import numpy as np
import pytest

FLT_MAX = 3.4028234663852886e38
MAX_POLY = 8


def f32(x):
    return struct.unpack("f", struct.pack("f", x))[0]


def bits(x):
    return struct.pack("f", x)


def sequential(vals):   # b2FindMaxSeparation's edge loop (mrp_world.h find_max_separation)
    best, max_sep = 0, -FLT_MAX
    for i, v in enumerate(vals):
        if v > max_sep:
            max_sep, best = v, i
    return best, max_sep


def grouped(vals, G):   # find_max_separation_grp
    lanes = []
    for sub in range(G):
        best, max_sep = MAX_POLY, -FLT_MAX
        for i in range(sub, len(vals), G):
            if vals[i] > max_sep:
                max_sep, best = vals[i], i
        lanes.append([max_sep, best])
    m = 1
    while m < G:   # butterfly over xor masks, every lane updated from its partner's previous value
        prev = [list(x) for x in lanes]
        for sub in range(G):
            os, ob = prev[sub ^ m]
            ms, b = prev[sub]
            if ob < MAX_POLY and (b == MAX_POLY or os > ms or (os == ms and ob < b)):
                lanes[sub] = [os, ob]
        m <<= 1
    out = set()
    for ms, b in lanes:
        out.add((0 if b == MAX_POLY else b, bits(-FLT_MAX if b == MAX_POLY else ms)))
    assert len(out) == 1, "every lane of the group must hold the same result"
    return out.pop()


POOL = [f32(x) for x in (0.0, -0.0, 1.5, -1.5, 2.0, -FLT_MAX, FLT_MAX, math.inf, -math.inf, 0.25, -0.25)] + [math.nan]


@pytest.mark.parametrize("G", [2, 4, 8])
def test_grouped_edge_scan_equals_sequential(G):
    rng = random.Random(1234 + G)
    for _ in range(20000):
        n = rng.randint(1, MAX_POLY)
        vals = [rng.choice(POOL) for _ in range(n)]
        b, s = sequential(vals)
        assert grouped(vals, G) == (b, bits(s)), vals


def test_grouped_edge_scan_exhaustive_small():
    small = [f32(0.0), f32(-0.0), f32(1.0), -FLT_MAX, math.nan]
    for n in range(1, 5):
        for vals in itertools.product(small, repeat=n):
            b, s = sequential(list(vals))
            for G in (2, 4, 8):
                assert grouped(list(vals), G) == (b, bits(s)), (vals, G)


def exit_mask(done, dense=32, sparse=16):
    return sparse - 1 if done > dense else 3


@pytest.mark.parametrize("pairs", [False, True])
def test_sparse_exit_schedule_is_exact(pairs):
    """Every compare point has its snapshot exactly two sweeps earlier and an even remainder."""
    for iters in range(1, 400):
        snap_at = None
        k0 = 0
        if pairs and iters & 1:
            k0 = 1                      # an odd count runs its first sweep alone
        if (iters - k0) & 3 == 2:
            snap_at = k0                # the start is a snapshot point
        step = 2 if pairs else 1
        k = k0
        while k < iters:
            k += step
            if not pairs and (iters - k) & 1:
                continue                # the single-sweep loops check only at even remainders
            left, m = iters - k, exit_mask(k)
            if left & m == 0 and snap_at is not None:
                assert k - snap_at == 2, (iters, k, snap_at)
                assert (iters - k) % 2 == 0
            if left & m == 2:
                snap_at = k


# ----------------------------------------------------------------------------- branch-free block solver
def _block_sequential(x1, b, nmass0, nmass1, k1):
    """b2ContactSolver::SolveVelocityConstraints' 2-point block solver case loop (mrp_world.h
    vel_update_m, case by case): the first case that holds gives x; None = no case holds."""
    f = lambda v: f32(v)  # noqa: E731
    if x1[0] >= 0.0 and x1[1] >= 0.0:
        return x1
    x = (f(f(-nmass0) * b[0]), 0.0)
    vn2 = f(f(k1 * x[0]) + b[1])
    if x[0] >= 0.0 and vn2 >= 0.0:
        return x
    x = (0.0, f(f(-nmass1) * b[1]))
    vn1 = f(f(k1 * x[1]) + b[0])
    if x[1] >= 0.0 and vn1 >= 0.0:
        return x
    if b[0] >= 0.0 and b[1] >= 0.0:
        return (0.0, 0.0)
    return None


def _block_selects(x1, b, nmass0, nmass1, k1):
    """The branch-free form (MRP_VEL_BFREE): all cases evaluated, picked by selects, one 'ok' mask."""
    f = lambda v: f32(v)  # noqa: E731
    x2 = f(f(-nmass0) * b[0]); v2 = f(f(k1 * x2) + b[1])
    x3 = f(f(-nmass1) * b[1]); v3 = f(f(k1 * x3) + b[0])
    c1 = x1[0] >= 0.0 and x1[1] >= 0.0
    c2 = x2 >= 0.0 and v2 >= 0.0
    c3 = x3 >= 0.0 and v3 >= 0.0
    c4 = b[0] >= 0.0 and b[1] >= 0.0
    xs = (x1[0] if c1 else (x2 if c2 else 0.0), x1[1] if c1 else (0.0 if c2 else (x3 if c3 else 0.0)))
    return xs if (c1 or c2 or c3 or c4) else None


def test_branch_free_block_solver_equals_case_loop():
    """Same impulse bits (signed zeros included) or the same 'no solution' for random, signed-zero,
    NaN, infinite and subnormal inputs of the case tests."""
    rng = random.Random(9)
    special = [0.0, -0.0, 1e-45, -1e-45, float("nan"), float("inf"), -float("inf"), 1.0, -1.0, 3.0e38]
    def val():
        return rng.choice(special) if rng.random() < 0.3 else f32(rng.uniform(-2, 2) * 10 ** rng.randint(-6, 3))
    for _ in range(200000):
        x1, b = (val(), val()), (val(), val())
        nm0, nm1, k1 = f32(abs(val())), f32(abs(val())), val()
        s = _block_sequential(x1, b, nm0, nm1, k1)
        t = _block_selects(x1, b, nm0, nm1, k1)
        assert (s is None) == (t is None), (x1, b, nm0, nm1, k1)
        if s is not None:
            assert bits(s[0]) + bits(s[1]) == bits(t[0]) + bits(t[1]), (x1, b, nm0, nm1, k1, s, t)


# ----------------------------------------------------------------------------- paired-slot schedule
def test_dual_schedule_keeps_every_body_in_sequential_order():
    """b2o_dual_schedule (the paired-update model of the 3-block accounting, oracle/b2_oracle.c):
    replaying its slots must give every dynamic body the same sequence of updates, and every contact
    its sweeps in order, as the Gauss-Seidel stream; a slot's two updates never share a dynamic body
    and have one point count."""
    import ctypes

    from oracle.oracle import lib
    L = lib()
    L.b2o_dual_schedule.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_int] * 2 + [ctypes.c_void_p, ctypes.c_int]
    L.b2o_dual_schedule.restype = ctypes.c_int
    rng = random.Random(5)
    arr = lambda v: (ctypes.c_int * len(v))(*v)  # noqa: E731
    for _ in range(300):
        nb, nc, D = rng.randint(2, 6), rng.randint(2, 8), rng.choice((1, 2, 3, 14))
        dyn = [1] * (nb - 1) + [0]                          # the last body static (a wall)
        ia = [rng.randrange(nb - 1) for _ in range(nc)]
        ib = [rng.randrange(nb) for _ in range(nc)]
        ib = [b if b != a else nb - 1 for a, b in zip(ia, ib)]
        pc = [rng.randint(1, 2) for _ in range(nc)]
        out = (ctypes.c_ubyte * 4096)()
        ns = L.b2o_dual_schedule(nc, arr(ia), arr(ib), arr(dyn), arr(pc), D, 16, out, 4096)
        assert 0 < ns <= nc * D
        # sequential: per body, the list of contact indices that update it, sweep by sweep
        seq = {b: [i for _ in range(D) for i in range(nc) if dyn[b] and b in (ia[i], ib[i])] for b in range(nb)}
        got = {b: [] for b in range(nb)}
        sweeps_run = [0] * nc
        n_upd = 0
        for t in range(ns):
            u, v = out[t] & 15, out[t] >> 4
            upd = [u] if u == v else [u, v]
            if len(upd) == 2:
                assert pc[u] == pc[v]
                assert not ({b for b in (ia[u], ib[u]) if dyn[b]} & {b for b in (ia[v], ib[v]) if dyn[b]})
            for i in upd:
                sweeps_run[i] += 1
                n_upd += 1
                for b in {ia[i], ib[i]}:
                    if dyn[b]:
                        got[b].append(i)
        assert n_upd == nc * D and sweeps_run == [D] * nc
        assert got == seq


def test_fixed_angle_stays_positive_zero():
    """The position passes' rotation memo (mrp_world.h RotMemo / UniMemo) answers an angle whose bits
    are +0 with b2Rot::Set(+0) = {+0, 1} without a lookup: a body with invI = 0 whose angle is +0 keeps
    the bit pattern +0 through every point update (a - 0 * x and a + 0 * x, float32) for every finite
    x, so the agents and walls of v0 / Heavy-v0 take that answer at every point; an infinite or NaN x
    makes it NaN (then rot() of it, as the reference's b2Rot::Set).  The round-6 ONE_ROT form built
    on the same property (profiles/r6_one_rot.patch) was measured and dropped."""
    rs = np.random.RandomState(3)
    bits = np.r_[rs.randint(0, 2 ** 32, 200000, dtype=np.uint64).astype(np.uint32),
                 np.array([0, 0x80000000, 1, 0x80000001, 0x7f7fffff, 0xff7fffff, 0x00800000, 0x80800000], np.uint32)]
    x = bits.view(np.float32)
    zero, izero = np.float32(0.0), np.float32(0.0)   # the angle +0 and invI = +0
    with np.errstate(invalid="ignore", over="ignore"):
        sub = zero - izero * x     # aA -= iA * cross(rA, P)
        add = zero + izero * x     # aB += iB * cross(rB, P)
    fin = np.isfinite(x)
    assert (sub[fin].view(np.uint32) == 0).all() and (add[fin].view(np.uint32) == 0).all()
    assert np.isnan(sub[~fin]).all() and np.isnan(add[~fin]).all()


def test_rot_fast_end_is_glibc_branch_point():
    """0x42f00000, the bits of 120.0f: the device's rot() keeps its straight-line rot_fast result
    exactly when abstop12(y) < abstop12(120.0f), i.e. when the |y| bit pattern is below 0x42f00000
    (NaN and infinities above it), and replaces it through glibc's other branches otherwise."""
    assert int(np.float32(120.0).view(np.uint32)) == 0x42F00000
    rs = np.random.RandomState(5)
    b = rs.randint(0, 2 ** 32, 500000, dtype=np.uint64).astype(np.uint32)
    abstop12 = (b >> 20) & 0x7FF
    assert np.array_equal(abstop12 < 0x42F, (b & 0x7FFFFFFF) < 0x42F00000)
