"""Build libmrp.so in-tree with hipcc for gfx950 (``python -m gym_puzzles_amd.build``).

Numerics flags are part of the contract: -ffp-contract=off (no FMA contraction, so float32
expressions round exactly like the box2d-py engine), no fast-math, f32 denormals kept,
correctly rounded f32 divide/sqrt.

Each env id's lane kernels are their own translation unit (csrc/mrp_env<E>.hip), so the units
compile in parallel and are linked into one shared library.
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libmrp.so")
N_ENVS = 23   # csrc/mrp_config.h N_ENVS: one translation unit per env id
SOURCES = ([os.path.join(CSRC, "mrp_kernels.hip"), os.path.join(CSRC, "mrp_tables.cpp"), os.path.join(CSRC, "mrp_norm.hip")]
           + [os.path.join(CSRC, f"mrp_env{e}.hip") for e in range(N_ENVS)])
DEPS = SOURCES + [os.path.join(CSRC, f) for f in ("mrp_math.h", "mrp_config.h", "mrp_world.h", "mrp_env.h", "mrp_tables.h",
                                                  "mrp_ops.h", "mrp_lane.h", "mrp_render.h")] + [
    os.path.join(HERE, "..", "include", "mrp.h"), os.path.abspath(__file__)]
# Per-unit flags.  The 3-block config (env 4, islands of 5-8 contacts) keeps its lanes-path sweep /
# pass loops as functions of their own, scheduled for ILP: the machine scheduler then drops the
# lanes-path update's s_nop wait states from about 40 to 17, +5.7 % env-steps/s in the driver window
# and +6.6 % at steps 21-220 (A/B, profiles/r3g_ab_scheduler.txt).  For v0 the same build gives
# +1.5 % in the driver window but -2.7 % at steps 21-220 (a call per island solve), so v0 keeps the
# inlined form.  Heavy-v0 (env 1, 5 agents): +1.4 % / +2.0 % (profiles/r3g_ab_scheduler.txt).
# Round 4 (profiles/r4_ab_unit_flags.txt): Heavy-v0 keeps the max-ilp scheduler with the loops
# inlined (+3.3 % in the driver window, +2.3 % at steps 21-220, PMC traffic 80.7 -> 49.4 MB per
# launch: no call-site register saves), while the 3-block config loses 5 % that way and keeps its
# loops out of line; v0 and v3 run the lanes-path sweeps two per loop trip (-DMRP_LANES_PAIRS=1:
# v0 +1.8 % / +0.7 %, v3 +0.5 %; Heavy-v0 -3 %, 3-block -0.3 %, so those keep one per trip).
_MAX_ILP = ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]
_ILP_LOOPS = ["-DMRP_SOLVE_NOINLINE_LANES"] + _MAX_ILP
_LANES_PAIRS = ["-DMRP_LANES_PAIRS=1"]
# v2 moves its live contact slots in 16-B granules (-DMRP_CONTACT_GRANULES=1): +2.5 % at the same
# traffic; for v0 / v3 the granules measured level in time and +16 % in traffic, so they move words
# (profiles/r4_ab_contact_granules.txt).
# v2 also takes the max-ilp scheduler on its inlined k_step (+3.2 % in the driver window, +3.0 % at
# steps 21-220; on v0 -0.2 % and on v3 -1.5 %, so those keep the default scheduler;
# profiles/r4_ab_max_ilp.txt).
_GRANULES = ["-DMRP_CONTACT_GRANULES=1"]
# v0 and v3 run under LLVM's iterative-ilp scheduler: v0 +4.4 % in the driver window and +4.8 % at
# steps 21-220, v3 +4.9 % / +4.4 %; Heavy-v0 -2 %, the 3-block config -1.7 % and v2 -2.5 % (against
# max-ilp) under it, so those keep their choices (profiles/r4_ab_sched_iterative_ilp.txt).
_ITER_ILP = ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"]
# Round 5 (profiles/r5_ab_bfree_xw.txt): v2 and the 3-block config pick the block solver's case
# without a chain of case tests (MRP_VEL_BFREE, with the two-ballot case test and the tangent speed as
# a cross product): their slowest lane-steps replayed alone +0.8 % / +3.3 %, bitwise; v0 -0.1 % (the
# selects and ballots add to every two-point update what the saved case tests take off), so v0 keeps
# the case loop; Heavy-v0 -1.0 % and v3 -4.9 % (profiles/r5_ab_bfree_env1_env5.txt) keep it too.
# With the "any case holds" test as per-lane selects as well (round 5's MRP_VEL_BFREE=2: the impulse applied
# unconditionally, each output selected, no ballot -> branch on the chain): v2 +2.8 % / +2.5 %,
# 3-block +2.4 % / +2.6 % (slowest lane-steps / driver window) over the ballot form; v0 +1.1 % in the
# driver window but -5 % over a whole episode (profiles/r5_ab_bfree2.txt), so v0 keeps the case loop.
_BFREE = ["-DMRP_VEL_BFREE=1", "-DMRP_VEL_PICK2=1", "-DMRP_VEL_VTCROSS=1"]
# v0 makes the values its step needs late (the state store's per-thread offsets, the TOI phase's
# zeroes) where they are used (-DMRP_FRESH_REGS=1): VGPR spills 14 -> 4, scratch 48 -> 16 B per
# thread, PMC traffic 30.9 -> 23.2 MB per launch; driver window -0.4 %, steps 21-220 -0.2 %, whole
# episode +0.7 % (profiles/r5_windows_traffic_fresh.txt).  Round 6 adds the thread id made opaque per
# island and TOI pass (refresh_tid): the round-6 code had brought v0 back to 14 spill stores at entry
# (PMC traffic 37.0 MB per launch); with it 4 (27.6 MB), driver window +0.4 % (profiles/r6_final_ab.txt).
# On Heavy-v0 / v2 / the 3-block unit it measured +0.4 / -0.5 / -0.9 % (profiles/r6_fresh_more_ab.txt).
_FRESH = ["-DMRP_FRESH_REGS=1"]
# v0 takes the branch-free selection (selects form) on its lanes path only (3+ contacts; the one- and
# two-contact register paths keep the case loop).  Round 6 re-measured it and round 5's two-ballot case
# test + cross-product tangent speed (MRP_VEL_PICK2 / MRP_VEL_VTCROSS) on all four windows, interleaved
# on one box (profiles/r6_windows_ab_v0.txt; driver window / steps 21-220 / 501-700 / whole episode
# against round 5's library): without PICK2_VT +0.9 / +0.7 / +0.7 / +1.3 %, without BFREE_LANES
# -0.6 / -0.4 / -0.1 / +0.1 %, without both -1.8 / -0.5 / +1.2 / +1.1 %.  So v0 keeps BFREE_LANES and
# drops PICK2_VT (it bought the driver window with the whole episode, DESIGN.md's rule).
_BFREE_LANES = ["-DMRP_VEL_BFREE=1", "-DMRP_VEL_BFREE_LANES=1"]
# v3 has the same spill pattern under the iterative-ilp schedule (14 VGPR spills -> 4): PMC traffic
# 30.8 -> 23.6 MB per launch, slowest lane-steps +0.7 %, driver window level (profiles/r5_ab_v3_fresh.txt).
# Round 6 (profiles/r6_bfree_paths_ab.txt, three interleaved rounds): the selects form on the lanes path
# only gives v3 +1.0 % (slowest lane-steps alone and driver window), so v3 takes BFREE_LANES; Heavy-v0
# +0.4 % with it (within the spread) keeps the case loop; on the register paths only (where v3's TOI
# sub-step solve runs) v3 measured -1.3 % / -1.5 %.
# v0 and v3 keep all 4096 lanes of a GPU resident: 4 waves per SIMD (a 128-VGPR budget, 54 VGPR spills).
# Their driver window is bounded by the slowest lane-step, their steady state by residency: at 4 waves
# v0's driver window is level (-0.3 / +0.2 %) and steps 21-220 / 501-700 / the whole episode gain
# +1.1 / +1.4 / +6.1 %; v3 +2.1 / +2.5 / +2.0 % (driver window / 501-700 / whole episode).  At 2 waves
# v0's steady state lost 7 % (profiles/r6_waves_ab.txt).  Round 3 had chosen 3 waves on the driver window
# alone (level) and the spills' traffic.
_W4 = ["-DMRP_STEP_WAVES_PER_EU=4"]
UNIT_FLAGS = {"mrp_env0.hip": _LANES_PAIRS + _ITER_ILP + _FRESH + _BFREE_LANES + _W4, "mrp_env1.hip": _MAX_ILP,
              "mrp_env2.hip": _GRANULES + _MAX_ILP + _BFREE, "mrp_env4.hip": _ILP_LOOPS + _BFREE,
              "mrp_env5.hip": _LANES_PAIRS + _ITER_ILP + _FRESH + _BFREE_LANES + _W4}
# -fno-slp-vectorize: the serial solver chains are latency-bound; packing pairs of f32 ops into
# v_pk_* costs operand-shuffling moves on the dependency chain (measured +2-3 % env-steps/s off)
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
         "-fno-gpu-flush-denormals-to-zero", "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-strict-aliasing",
         "-fno-slp-vectorize", "-fPIC", "-Wno-pass-failed"]


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.exists(c) or c == "hipcc"):
            return c
    return "hipcc"


def up_to_date() -> bool:
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(d) <= t for d in DEPS if os.path.exists(d))


def build(force: bool = False, verbose: bool = False, out: str = OUT, defines=(), jobs: int | None = None,
          only_envs=None) -> str:
    """Build libmrp.so (or a diagnostic variant with extra -D defines into ``out``).

    ``only_envs`` (A/B libraries): compile only those env units (plus the small shared units) and link
    the other env units' objects of the default build, which must exist; each env unit is
    self-contained, so the variant differs from the default library only in the listed envs."""
    if not force and out == OUT and up_to_date():
        return out
    objdir = os.path.join(HERE, "build", os.path.basename(out) + ".obj")
    os.makedirs(objdir, exist_ok=True)
    dflags = [f"-D{d}" for d in defines]
    objs = [os.path.join(objdir, os.path.basename(s) + ".o") for s in SOURCES]
    todo = list(range(len(SOURCES)))
    if only_envs is not None:
        assert out != OUT, "only_envs builds a variant library, never the default one"
        keep = {f"mrp_env{e}.hip" for e in only_envs}
        base = os.path.join(HERE, "build", os.path.basename(OUT) + ".obj")
        todo = [i for i, s in enumerate(SOURCES) if "mrp_env" not in s or os.path.basename(s) in keep]
        # the reused objects must have been compiled from the current sources and headers: an env
        # unit built before a shared header changed would mix two layouts in one A/B library
        # (MRP_ALLOW_STALE_UNITS=1 accepts it for an A/B of the listed envs when the edit leaves the
        # LaneState / EnvOps layout unchanged; mrp_create still checks each unit's compiled dims)
        newest_dep = max(os.path.getmtime(d) for d in DEPS if os.path.exists(d) and d.endswith((".h", ".hip", ".cpp")))
        for i, s in enumerate(SOURCES):
            if i not in todo:
                objs[i] = os.path.join(base, os.path.basename(s) + ".o")
                if not os.path.exists(objs[i]):
                    raise FileNotFoundError(f"{objs[i]}: build the default library first")
                if os.path.getmtime(objs[i]) < newest_dep and not os.environ.get("MRP_ALLOW_STALE_UNITS"):
                    raise RuntimeError(f"{objs[i]} is older than a source or header it depends on: rebuild the default "
                                       "library (python -m gym_puzzles_amd.build) before a variant")

    # A/B only: extra compiler flags for a variant library (never the default one)
    extra = os.environ.get("MRP_EXTRA_FLAGS", "").split() if out != OUT else []

    headers = [d for d in DEPS if d.endswith(".h")]
    newest_header = max(os.path.getmtime(d) for d in headers if os.path.exists(d))

    def compile_one(i: int) -> None:
        unit = UNIT_FLAGS.get(os.path.basename(SOURCES[i]), []) if not extra else []
        cmd = [hipcc()] + FLAGS + unit + extra + dflags + ["-c", SOURCES[i], "-o", objs[i]]
        # incremental: an object newer than its source and every header, built with the same command
        # line (recorded beside it), is kept; the env units include every header, so a header edit
        # rebuilds them all, while an edit of mrp_kernels.hip alone rebuilds that unit only
        stamp = objs[i] + ".cmd"
        line = " ".join(cmd)
        if not force and os.path.exists(objs[i]) and os.path.exists(stamp):
            t = os.path.getmtime(objs[i])
            with open(stamp) as f:
                same = f.read() == line
            if same and t >= os.path.getmtime(SOURCES[i]) and t >= newest_header:
                return
        if verbose:
            print(line, flush=True)
        subprocess.run(cmd, check=True)
        with open(stamp, "w") as f:
            f.write(line)

    # slowest units first; each hipcc is single-threaded, so one job per core
    jobs = jobs or max(1, min(len(SOURCES), os.cpu_count() or 1, int(os.environ.get("MAX_JOBS", "16"))))
    order = sorted(todo, key=lambda i: "mrp_env" not in SOURCES[i])
    with ThreadPoolExecutor(jobs) as ex:
        list(ex.map(compile_one, order))
    cmd = [hipcc()] + FLAGS + ["-shared"] + objs + ["-o", out + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    if "--stamps" in sys.argv:   # diagnostic per-phase timing build (tools/phase_profile.py; --variant builds fewer units)
        print(build(verbose=True, out=os.path.join(HERE, "libmrp_stamps.so"), defines=("MRP_STAMPS",)))
    elif "--progress" in sys.argv:   # diagnostic hang-localisation build (tools/hang_probe.py)
        print(build(verbose=True, out=os.path.join(HERE, "libmrp_progress.so"), defines=("MRP_PROGRESS",)))
    elif "--variant" in sys.argv:   # A/B library: python -m gym_puzzles_amd.build --variant OUT.so E [E ...] [-DNAME ...]
        i = sys.argv.index("--variant")
        args = sys.argv[i + 2:]
        envs = [int(a) for a in args if not a.startswith("-D")]
        defs = [a[2:] for a in args if a.startswith("-D")]
        print(build(verbose=True, out=os.path.abspath(sys.argv[i + 1]), defines=defs, only_envs=envs))
    else:
        print(build(force="--force" in sys.argv, verbose=True))   # --force: recompile every unit
