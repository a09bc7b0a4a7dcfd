#!/usr/bin/env python3
"""Benchmark: env-steps/sec of the MI355X-native MultiRobotPuzzle step (BASELINE.json metric).

Workload (BASELINE.json configs[1]): MultiRobotPuzzle-v0, 4096 lanes (independent worlds) per
GPU, synthetic random actions generated on device (counter RNG keyed by global lane and step),
gym TimeLimit + done -> on-device auto-reset inside the timed loop (as SB3's VecEnv would).
A "step" is one k_step launch advancing every lane of every rank by one env step.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--env ID] [--lanes L]

For N > 1 launch one process per GPU (torch.distributed.run); lanes shard contiguously
(rank r owns global lanes [r*L, (r+1)*L)), per-lane trajectories are independent of N, and
each step ends with one gather of (obs, reward, done) to rank 0 (the policy rank).
Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

ENV_NAMES = {0: "MultiRobotPuzzle-v0", 1: "MultiRobotPuzzleHeavy-v0", 2: "MultiRobotPuzzle-v2",
             3: "MultiRobotPuzzleHeavy-v2", 4: "MultiRobotPuzzleHeavy-v2-3block", 5: "MultiRobotPuzzle-v3",
             6: "MultiRobotPuzzle-v3-heavy"}
# Algorithmic HBM bytes per env-step: mutable per-lane state read+written
# once per step plus I/O; shared geometry/mass tables excluded.
ALGO_BYTES = {0: 1657, 1: 3547, 2: 3613, 3: 3613, 4: 6085, 5: 1653, 6: 1653}   # v3: v0's lane state, 27-float obs
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md chip table (spec)
# the gym-style single env of each config (make() id and constructor arguments) for the drop-in diagnostic
SINGLE_ENV_MAKE = {0: ("MultiRobotPuzzle-v0", {}), 1: ("MultiRobotPuzzleHeavy-v0", {}), 2: ("MultiRobotPuzzle-v2", {}),
                   3: ("MultiRobotPuzzleHeavy-v2", {}), 4: ("MultiRobotPuzzleHeavy-v2-3block", {}),
                   5: ("MultiRobotPuzzle-v3", {}), 6: ("MultiRobotPuzzle-v3", {"heavy": True})}


def host_cpus() -> dict:
    """The host CPUs this process may use: nproc, the affinity mask, the cgroup CPU quota and
    OMP_NUM_THREADS, and the resulting allotment.  On the GPU box `nproc` and the affinity mask
    show the whole machine while the job's share is smaller, so the allotment is the cgroup quota
    when one is set, else OMP_NUM_THREADS when the launcher set it, else the affinity mask."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            with open(path) as f:
                parts = f.read().split()
            if path.endswith("cpu.max") and parts and parts[0] != "max":
                quota = float(parts[0]) / float(parts[1])
            elif path.endswith("quota_us") and parts and int(parts[0]) > 0:
                with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                    quota = int(parts[0]) / float(f.read().split()[0])
            if quota:
                break
        except (OSError, ValueError, IndexError):
            continue
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or None
    if quota:
        allot, rule = max(1, min(aff, int(quota + 0.5))), "cgroup cpu quota"
    elif omp:
        allot, rule = max(1, min(aff, omp)), "OMP_NUM_THREADS (no cgroup quota)"
    else:
        allot, rule = aff, "affinity mask (no cgroup quota, no OMP_NUM_THREADS)"
    return {"nproc": os.cpu_count(), "affinity": aff, "cgroup_quota_cpus": quota, "omp_num_threads": omp,
            "allotted": allot, "rule": rule}


def _oracle_rate(variant: str, env_id: int, lanes: int, skip: int, steps: int, seed: int, threads: int, target_s: float,
                 max_reps: int) -> dict:
    """Time one oracle build (oracle/Makefile variant) on `lanes` lanes x steps skip+1 .. skip+steps
    after spawn, the same counter-RNG workload as the GPU line; repetition r uses seed + r (r = 0 is
    exactly the GPU's lanes), repeated until about `target_s` seconds of timed work."""
    from gym_puzzles_amd.spawn import draw_bounds
    from oracle.oracle import batch_run  # test infrastructure: baseline leg only
    bounds = draw_bounds(env_id)
    # one untimed repetition first: the first pass over fresh worlds pays page faults and allocator
    # growth (4-5x slower on the first call in a process), which is not the step's cost
    batch_run(env_id, lanes, steps, seed, bounds, threads=threads, skip=skip, variant=variant)
    n_tot, dt_tot, reps, rep0 = 0, 0.0, 0, None
    while reps < max_reps and (reps == 0 or dt_tot < target_s):
        n, dt = batch_run(env_id, lanes, steps, seed + reps, bounds, threads=threads, skip=skip, variant=variant)
        n_tot, dt_tot, reps = n_tot + n, dt_tot + dt, reps + 1
        if rep0 is None:
            rep0 = n / max(dt, 1e-9)
    return {"value": n_tot / max(dt_tot, 1e-9), "seconds": dt_tot, "env_steps": n_tot, "reps": reps,
            "seeds": [seed, seed + reps - 1], "first_rep_value": rep0}


def cpu_baseline(env_id: int, lanes: int, seed: int, skip: int, steps: int, episode: bool = True,
                 target_s: float = 8.0) -> dict:
    """The CPU baseline (cpu_baseline in the JSON line), timed like for like with the GPU line:
    the C restatement of the step (oracle/, kind "port": pybox2d cannot run here or on the GPU
    box) built WITHOUT the work model (oracle/Makefile libmrp_oracle_port.so: the Box2D algorithm,
    all 180 velocity sweeps as b2Island::Solve runs them), on all allotted host cores, over the
    GPU line's own window -- the same lanes, steps skip+1 .. skip+steps after spawn, the same
    counter-RNG spawns and actions, auto-reset -- repeated over seeds to ~target_s seconds.
    Beside it (never `value`): the same build over one whole episode; the early-exit port
    (libmrp_oracle_early.so: the device's exact period-1/2 exit of the velocity sweeps, same bits)
    on the same window and episode, so GPU / CPU separates the hardware from that algorithmic
    saving; and one lane on one core (BASELINE.json configs[0])."""
    from gym_puzzles_amd.spawn import draw_bounds
    from oracle.oracle import batch_run, build_kind, lib  # test infrastructure: baseline leg only
    cpus = host_cpus()
    threads = cpus["allotted"]
    port = _oracle_rate("port", env_id, lanes, skip, steps, seed, threads, target_s, 400)
    early = _oracle_rate("early", env_id, lanes, skip, steps, seed, threads, target_s / 2, 400)
    out = {"value": port["value"], "unit": "env-steps/s", "cores": threads, "kind": "port",
           "sample": f"{ENV_NAMES[env_id]}: {lanes} lanes x steps {skip + 1}-{skip + steps} after spawn (the GPU line's "
                     f"window; device-RNG actions and spawns, auto-reset), {port['reps']} repetitions over seeds "
                     f"{port['seeds'][0]}-{port['seeds'][1]} (seed {seed} = the GPU's lanes), {threads} OpenMP threads, "
                     f"{port['seconds']:.1f} s timed; build oracle/build/libmrp_oracle_port.so ({build_kind('port')})",
           "window": port, "host_cpus": cpus,
           "early_exit_port": dict(early, build=build_kind("early"),
                                   note="same window and bits; velocity sweeps stop at the device's exact early exit")}
    bounds = draw_bounds(env_id)
    T = lib("port").or_max_episode_steps(env_id)
    if episode:
        eps = {}
        for v in ("port", "early"):
            n, dt = batch_run(env_id, lanes, T, seed, bounds, threads=threads, variant=v)
            eps[v] = {"steps": T, "value": n / max(dt, 1e-9), "seconds": dt}
        out["whole_episode"] = eps
    # one lane on one core: whole episodes over seeds, about 3 s
    n1, dt1, r1 = 0, 0.0, 0
    while dt1 < 3.0 and r1 < 200:
        n, dt = batch_run(env_id, 1, T, seed + r1, bounds, threads=1, variant="port")
        n1, dt1, r1 = n1 + n, dt1 + dt, r1 + 1
    out["single_lane_1core"] = {"value": n1 / max(dt1, 1e-9), "unit": "env-steps/s", "cores": 1,
                                "sample": f"1 lane x {T} steps (one whole episode) x {r1} seeds of the same workload, "
                                          f"port build, 1 thread, {dt1:.1f} s (BASELINE.json configs[0]: 1 env on the CPU)"}
    return out


def single_env_rate(env_id: int, steps: int = 300, seeds=(0, 1, 2, 3)) -> dict:
    """Diagnostic (never `value`): the gym-style drop-in path, `make(id)` then env.step(a) with host
    numpy actions - one lane per call, PCIe round trip included (what train.py's DummyVecEnv drives).

    The step is one 1-lane k_step launch, i.e. one lane's serial chain, so its time follows the
    episode: an agent pressed against the block runs the 180 velocity sweeps and the position passes,
    a free one does not.  The reference's reset draws its spawn from the global np.random, which an
    unseeded run leaves at a random state, and that made single runs bimodal (36-39 us against
    48-61 us in round 5).  Each timed episode here starts from np.random.seed(s) for the listed seeds
    (the same spawn and actions every run), and the line reports their mean with the per-seed times
    and the lane's touching contacts and position iterations per step."""
    from gym_puzzles_amd import make
    name, kw = SINGLE_ENV_MAKE[env_id]
    per = []
    for sd in seeds:
        np.random.seed(sd)   # the reference's spawn RNG (global np.random)
        env = make(name, **kw)
        env.unwrapped.seed(sd)
        env.reset()
        rs = np.random.RandomState(sd)
        acts = rs.uniform(-1, 1, size=(steps + 20, env.action_space.shape[0])).astype(np.float32)
        for k in range(20):
            _, _, d, _ = env.step(acts[k])
            if d:
                env.reset()
        c0 = env.unwrapped._b.counters_ex()
        t0 = time.perf_counter()
        for k in range(steps):
            _, _, d, _ = env.step(acts[20 + k])
            if d:
                env.reset()
        dt = time.perf_counter() - t0
        c1 = env.unwrapped._b.counters_ex()
        env.close()
        per.append({"seed": sd, "us_per_step": dt / steps * 1e6,
                    "touching_contacts_per_step": (c1["touching_contacts"] - c0["touching_contacts"]) / steps,
                    "position_iterations_per_step": (c1["position_iterations"] - c0["position_iterations"]) / steps})
    us = float(np.mean([p["us_per_step"] for p in per]))
    return {"env_steps_per_s": 1e6 / us, "us_per_step": us, "steps": steps, "seeds": list(seeds), "per_seed": per,
            "path": f"gym_puzzles_amd.make('{name}'{''.join(f', {k}={v!r}' for k, v in kw.items())}).step(): "
                    "1-lane kernel, actions and outputs through the ctx's pinned host buffer"}


def load_valu(env_id: int, lanes: int, first: int, last: int, seed: int, kern_ms: float):
    """roofline.valu: the oracle op-count model of exactly this workload (tools/roofline_model.py ->
    profiles/r3_valu_latency.json, keyed by env, lanes, timed step window and seed) over the live
    kernel_ms; None when the table has no entry for this run."""
    path = os.path.join(HERE, "profiles", "r3_valu_latency.json")
    try:
        with open(path) as f:
            m = json.load(f)[f"{env_id}:{lanes}:{first}:{last}:{seed}"]
    except (OSError, ValueError, KeyError):
        return None
    peak = m["constants"]["valu_peak_flops"]
    ach = m["flops_per_launch"] / (kern_ms * 1e-3)
    return {"achieved": ach / 1e12, "peak": peak / 1e12, "unit": "TFLOP/s", "frac": ach / peak,
            "flops_per_launch": m["flops_per_launch"],
            "source": "oracle op counts of this exact workload (tools/roofline_model.py, profiles/r3_valu_latency.json)"}


ISSUE_TABLE = "r6_issue_roofline.json"


def load_issue(env_id: int, lanes: int, first: int, last: int, seed: int, kern_ms: float):
    """roofline.issue: the instruction-issue floor of the lane-steps that set each launch's duration.
    Each timed launch's slowest lane-step was captured (tools/issue_capture.py) and replayed alone under
    rocprofv3 (tools/issue_replay.py): SQ_INSTS counts its executed instructions, and a lone wave issues
    one instruction per 4 cycles of any type (MI355X_MICROARCH.md, 'vector-instruction ISSUE cost'), so
    its floor is 4 x SQ_INSTS cycles at the in-kernel clock (s_memtime / s_memrealtime of the stamps
    build).  frac = floor / the live kernel_ms.  `lone_wave_ms` is the same lane-step's measured
    duration alone (kernel trace): the model of the launch (the launch lasts as long as its slowest
    lane), whose gap to the floor is latency (dependent chains, LDS and memory waits) and whose gap
    to kernel_ms is co-resident waves.  None when profiles/ISSUE_TABLE has no entry."""
    path = os.path.join(HERE, "profiles", ISSUE_TABLE)
    try:
        with open(path) as f:
            m = json.load(f)[f"{env_id}:{lanes}:{first}:{last}:{seed}"]
    except (OSError, ValueError, KeyError):
        return None
    floor_ms = m["issue_floor_us_mean"] * 1e-3
    lone_ms = m["lone_wave_duration_us_mean"] * 1e-3
    out = {"floor_ms": floor_ms, "kernel_ms": kern_ms, "frac": floor_ms / kern_ms,
           "lone_wave_ms": lone_ms, "lone_wave_over_kernel": lone_ms / kern_ms,
           "slowest_lane_instructions": m["slowest_lane_instructions_mean"],
           "in_kernel_clock_ghz": m["in_kernel_clock_ghz"],
           "source": f"profiles/{ISSUE_TABLE} (tools/issue_capture.py, issue_replay.py, issue_roofline.py)"}
    if "note" in m:
        out["note"] = m["note"]
    return out


def load_traffic(env_id: int, lanes: int):
    """HBM bytes per k_step launch from the committed rocprofv3 PMC pass (profiles/), or None."""
    path = os.path.join(HERE, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        e = d.get(str(env_id))
        if e and int(e.get("lanes", -1)) == lanes:
            return float(e["hbm_bytes_per_launch"])
    except (OSError, ValueError, KeyError):
        pass
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--env", type=int, default=0)
    ap.add_argument("--lanes", type=int, default=4096, help="lanes (worlds) per GPU")
    ap.add_argument("--seed", type=int, default=17)
    ap.add_argument("--no-gather", action="store_true", help="N>1: skip the per-step gather to rank 0")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="N>1: torch.distributed backend; nccl = RCCL over xGMI (the default), gloo = the same "
                         "code path with the packed [L, O+2] block staged through pinned host memory (runs "
                         "with several ranks on one GPU, where RCCL refuses duplicate devices)")
    ap.add_argument("--same-device", action="store_true",
                    help="N>1 rehearsal on one GPU: every rank uses device 0 (with --dist-backend gloo)")
    ap.add_argument("--force-collective", action="store_true",
                    help="run the distributed branch (init_process_group, per-step gather) even at WORLD_SIZE 1, so a "
                         "one-GPU box executes the RCCL gather on device tensors (launch under torch.distributed.run "
                         "--nproc-per-node 1)")
    ap.add_argument("--dump-gather", default="",
                    help="N>1 check: rank 0 saves every timed step's gathered (obs | reward | done) rows to this .npy")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--schedule", type=int, default=-1, help="mrp_set_schedule mode: 0 lane order, 1 costliest-first dispatch, 2 cost priority, 3 both; default: the library's per-env choice (mrp_create)")
    ap.add_argument("--time-every", type=int, default=0,
                    help="0 (default): one HIP event pair around all K timed launches on the kernel's stream, kernel_ms = "
                         "that time / K; N >= 1: also bracket every N-th launch (per-launch spread; each marker pair "
                         "costs the stream ~8 us, so this lowers `value`)")
    ap.add_argument("--single-env", type=int, default=300,
                    help="diagnostic: steps of the gym-style 1-lane make(id).step() path to time (0 = off; N=1 only)")
    ap.add_argument("--later-window", type=int, default=200,
                    help="diagnostic: also time this many steps starting near --later-start (0 = off; N=1 only)")
    ap.add_argument("--later-start", type=int, default=500)
    ap.add_argument("--episode", type=int, default=1,
                    help="diagnostic: also time one whole episode (TimeLimit steps from spawn, N=1 only; 0 = off)")
    ap.add_argument("--multi-step", type=int, default=10,
                    help="diagnostic: also time launches of K env steps (mrp_step_n_device) against single-step launches "
                         "over the same window (0/1 = off; N=1 only)")
    ap.add_argument("--multi-window", type=int, default=200, help="steps timed by the --multi-step diagnostic")
    ap.add_argument("--vecnormalize", action="store_true",
                    help="also run SB3 VecNormalize + Monitor statistics on the device every step (train.py:68,80-82)")
    args = ap.parse_args()
    if args.same_device and args.dist_backend != "gloo":
        ap.error("--same-device needs --dist-backend gloo (RCCL refuses two ranks on one device)")
    if args.same_device and int(os.environ.get("WORLD_SIZE", "1")) < 2:
        ap.error("--same-device is a rehearsal of N > 1 ranks on one GPU: launch 2+ ranks under torch.distributed.run")
    if args.force_collective and "WORLD_SIZE" not in os.environ:
        ap.error("--force-collective: launch under torch.distributed.run (WORLD_SIZE / MASTER_ADDR come from it)")

    import torch
    import torch.distributed as dist

    from gym_puzzles_amd import Batch
    from gym_puzzles_amd.dist import Shard, StepGather

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("for --gpus > 1 launch with torch.distributed.run --nproc-per-node N")
    distributed = world > 1 or args.force_collective
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU (libmrp has no CPU fallback)")
    gpu = 0 if args.same_device else local_rank
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    host_coll = distributed and args.dist_backend == "gloo"
    if distributed:
        if host_coll:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    cdev = torch.device("cpu") if host_coll else dev   # where the small control collectives run

    L = args.lanes
    b = Batch(args.env, L, device=gpu, seed=args.seed, lane_offset=rank * L)
    # a dedicated (non-NULL) stream shared by the library and torch, so the HIP events that
    # time k_step are recorded on the stream the kernel runs on
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    b.set_stream(stream.cuda_stream)
    b.set_auto_reset(True)
    if args.schedule >= 0:
        b.set_schedule(args.schedule)
    O = b.obs_dim
    obs = torch.zeros((L, O), dtype=torch.float32, device=dev)
    rew = torch.zeros(L, dtype=torch.float32, device=dev)
    done = torch.zeros(L, dtype=torch.uint8, device=dev)
    trunc = torch.zeros(L, dtype=torch.uint8, device=dev)
    status = torch.zeros(L, dtype=torch.uint8, device=dev)
    # one contiguous buffer per rank for the gather: [obs | reward | done] as float32
    gather = (StepGather(Shard(rank, world, L), O, dev, host_stage=host_coll, force_collective=args.force_collective)
              if distributed and not args.no_gather else None)
    dumps = [] if (args.dump_gather and rank == 0 and gather is not None) else None

    b.reset()   # device-RNG spawns for every lane (seeded by global lane id)
    norm = None
    if args.vecnormalize:
        from gym_puzzles_amd import DeviceVecNormalize
        norm = DeviceVecNormalize(L, O, gpu)
        term = torch.zeros((L, O), dtype=torch.float32, device=dev)
        nobs, nrew, nterm = torch.zeros_like(obs), torch.zeros_like(rew), torch.zeros_like(term)
        epr, epl = torch.zeros(L, dtype=torch.float64, device=dev), torch.zeros(L, dtype=torch.int32, device=dev)
        norm.reset(torch.from_numpy(b.obs).to(dev), nobs)

    def one_step():
        b.step_device(0, obs.data_ptr(), rew.data_ptr(), done.data_ptr(), trunc.data_ptr(), status.data_ptr(),
                      0 if norm is None else term.data_ptr())
        if norm is not None:
            norm.step(obs, rew, done, nobs, nrew, term, nterm, epr, epl)
        if gather is not None:
            gather(nobs if norm is not None else obs, nrew if norm is not None else rew, done)

    for _ in range(args.warmup):
        one_step()
    torch.cuda.synchronize(dev)
    ctr0 = b.counters_ex()   # the batch counters count from creation: the timed window is the difference

    K = args.steps
    # kernel_ms: k_step's mean launch duration over exactly the K timed launches.  When k_step is
    # the only work on the stream (no gather, no VecNormalize), one event pair around the K
    # launches gives it without markers between launches (stream-busy time / K, launch gaps
    # included, so kernel_ms <= ms_per_step); otherwise every launch is bracketed.  --time-every N
    # adds per-launch brackets on every N-th launch for the spread (diagnostic; costs `value`).
    alone = gather is None and norm is None
    TE = args.time_every if alone else 1
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) if TE and k % TE == 0 else None
          for k in range(K)]
    r0, r1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if distributed:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    r0.record(stream)
    for k in range(K):
        if ev[k] is not None:
            ev[k][0].record(stream)
        b.step_device(0, obs.data_ptr(), rew.data_ptr(), done.data_ptr(), trunc.data_ptr(), status.data_ptr(),
                      0 if norm is None else term.data_ptr())
        if ev[k] is not None:
            ev[k][1].record(stream)
        if norm is not None:
            norm.step(obs, rew, done, nobs, nrew, term, nterm, epr, epl)
        if gather is not None:
            gather(nobs if norm is not None else obs, nrew if norm is not None else rew, done)
            if dumps is not None:
                # an asynchronous copy on the stream (device buffer) or a host memcpy (host-staged):
                # no synchronising device -> host transfer in the timed loop; the JSON line is marked
                # (config.dump_gather) so its rate is never quoted as throughput
                dumps.append(gather.full.clone())
    r1.record(stream)
    torch.cuda.synchronize(dev)
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ev = [x for x in ev if x is not None]
    kts = np.array([s.elapsed_time(e) for s, e in ev]) if ev else None
    if alone and TE == 0:
        kern_ms = r0.elapsed_time(r1) / K
        timing = f"one HIP event pair on the kernel's stream around all {K} timed launches (stream-busy time / {K})"
    elif alone and TE > 1:
        kern_ms = r0.elapsed_time(r1) / K
        timing = (f"one HIP event pair on the kernel's stream around all {K} timed launches (stream-busy time / {K}, "
                  f"including the markers around every {TE}th launch)")
    else:
        kern_ms = float(np.mean(kts))
        timing = f"HIP events around each of the {K} timed k_step launches"
    # the run must not hide a broken lane: loop-guard faults and non-finite outputs are checked
    # over the timed window (status bit MRP_STATUS_NONFINITE marks a lane-step with NaN/inf)
    flt = b.faults()
    ctr1 = b.counters_ex()
    ctr_window = {k: ctr1[k] - ctr0[k] for k in ctr1}
    bad = {"lanes_with_loop_guard_fault": int(np.count_nonzero(flt)),
           "obs_finite": bool(torch.isfinite(obs).all().item()),
           "nonfinite_lane_steps": int(ctr_window["nonfinite_steps"])}
    if distributed:
        t = torch.tensor([elapsed, kern_ms, bad["lanes_with_loop_guard_fault"], 0 if bad["obs_finite"] else 1,
                          bad["nonfinite_lane_steps"]], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
        bad = {"lanes_with_loop_guard_fault": int(t[2]), "obs_finite": not bool(t[3]), "nonfinite_lane_steps": int(t[4])}
    checks_ok = bad["lanes_with_loop_guard_fault"] == 0 and bad["obs_finite"] and bad["nonfinite_lane_steps"] == 0

    ctr = {"timed_window": ctr_window, "since_creation": ctr1} if rank == 0 else {}
    # Diagnostics only (never `value`): the rate over a later window of the same episodes (every
    # lane spawned at step 0; the first tens of steps after a spawn carry most of the overlap
    # resolution, so a window's rate depends on where it sits).
    later = None
    if args.later_window > 0 and rank == 0 and not distributed:
        skip = max(0, args.later_start - (args.warmup + K))
        for _ in range(skip):
            one_step()
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        s0.record(stream)
        for _ in range(args.later_window):
            one_step()
        s1.record(stream)
        torch.cuda.synchronize(dev)
        first = args.warmup + K + skip + 1
        later = {"steps_after_spawn": [first, first + args.later_window - 1],
                 "env_steps_per_s": L * args.later_window / (s0.elapsed_time(s1) * 1e-3)}
    # Diagnostic only (never `value`): one whole episode from spawn to the TimeLimit reset, every
    # lane in lockstep as SB3's DummyVecEnv keeps them (v0 ends early only on puzzle completion):
    # the rate averaged over every phase of an episode.
    episode = None
    if args.episode and rank == 0 and not distributed:
        T = b.max_episode_steps
        b.reset()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        e0.record(stream)
        for _ in range(T):
            one_step()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        episode = {"steps": T, "env_steps_per_s": L * T / (e0.elapsed_time(e1) * 1e-3)}
    # Diagnostic (never `value`): K env steps per launch (mrp_step_n_device) against single-step
    # launches over the same window of the same trajectories (two batches, same seed): every step's
    # outputs are written either way, so the gap is what the per-step max-over-lanes tail costs.
    multi = None
    if args.multi_step > 1 and rank == 0 and not distributed and norm is None:
        Km, Tm = args.multi_step, args.multi_window
        Tm = max(Km, Tm // Km * Km)
        rates = {}
        for mode in ("single", "multi"):
            bm = Batch(args.env, L, device=local_rank, seed=args.seed + 1)
            bm.set_stream(stream.cuda_stream)
            bm.set_auto_reset(True)
            bm.reset()
            mo = torch.zeros((Km, L, O), dtype=torch.float32, device=dev)
            mr = torch.zeros((Km, L), dtype=torch.float32, device=dev)
            md = torch.zeros((Km, L), dtype=torch.uint8, device=dev)
            for _ in range(args.warmup):
                bm.step_device(0, mo.data_ptr(), mr.data_ptr(), md.data_ptr())
            m0, m1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize(dev)
            m0.record(stream)
            if mode == "single":
                for k in range(Tm):
                    bm.step_device(0, mo[k % Km].data_ptr(), mr[k % Km].data_ptr(), md[k % Km].data_ptr())
            else:
                for _ in range(Tm // Km):
                    bm.step_n_device(Km, 0, mo.data_ptr(), mr.data_ptr(), md.data_ptr())
            m1.record(stream)
            torch.cuda.synchronize(dev)
            rates[mode] = L * Tm / (m0.elapsed_time(m1) * 1e-3)
            bm.close()
        multi = {"steps_per_launch": Km, "steps_after_spawn": [args.warmup + 1, args.warmup + Tm],
                 "env_steps_per_s": rates["multi"], "single_step_launches_env_steps_per_s": rates["single"],
                 "ratio": rates["multi"] / rates["single"]}
    single = None
    if args.single_env > 0 and rank == 0 and not distributed:
        single = single_env_rate(args.env, args.single_env)
    if rank == 0:
        total_steps = world * L * K
        value = total_steps / elapsed
        algo_bytes = ALGO_BYTES[args.env] * L
        achieved = algo_bytes / (kern_ms * 1e-3) / 1e9
        traffic = load_traffic(args.env, L)
        valu = load_valu(args.env, L, args.warmup + 1, args.warmup + K, args.seed, kern_ms)
        issue = load_issue(args.env, L, args.warmup + 1, args.warmup + K, args.seed, kern_ms)
        line = {
            "metric": "env-steps/sec (whole node) at N envs/GPU",
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": elapsed / K * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32 (engine) + f64 (env arithmetic)",
            "data": "synthetic: device-RNG random actions, device-RNG spawns (reference draw ranges)",
            "config": {"workload": f"{ENV_NAMES[args.env]}, {L} lanes/GPU, random actions, auto-reset", "env_id": args.env,
                       "lanes_per_gpu": L, "global_lanes": world * L,
                       "parallelism": f"lane-sharded x{world}" + ("" if not distributed or args.no_gather else " + gather to rank 0/step"),
                       "collective": None if not distributed or args.no_gather else
                                     (args.dist_backend + (" (host-staged)" if host_coll else " (RCCL)")
                                      + (" forced at world size 1" if world == 1 else "")),
                       "dump_gather": bool(dumps is not None),
                       "devices": 1 if (world == 1 or args.same_device) else world,
                       "vecnormalize": bool(args.vecnormalize),
                       "dispatch": ("lane order" if args.schedule == 0 else f"mrp_set_schedule({args.schedule})") if args.schedule >= 0
                                   else "library default (costliest-first for Heavy-v0 / v3 beyond the resident waves, else lane order)"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic,
                         "kernel": "k_step", "kernel_ms": kern_ms,
                         "kernel_ms_timing": timing,
                         "algorithmic_bytes_per_launch": algo_bytes,
                         "limiter": "instruction issue of the slowest lane's wave (one instruction per 4 cycles, serial "
                                    "Gauss-Seidel chains: velocity sweeps, position passes, TOI) and its latency stalls; "
                                    "not HBM and not MFMA",
                         "note": "HBM fraction reported because the north star asks for it (SURVEY.md 8d)",
                         "valu": valu, "issue": issue},
            "checks": dict(bad, ok=checks_ok),
            "diagnostics": {"counters": ctr,
                            "timed_steps_after_spawn": [args.warmup + 1, args.warmup + K],
                            "kernel_ms_min_median_max": None if kts is None else
                            [float(kts.min()), float(np.median(kts)), float(kts.max())],
                            "later_window": later, "whole_episode": episode, "multi_step_launch": multi,
                            "single_env_drop_in": single},
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args.env, L, args.seed, args.warmup, K)
            cb = line["cpu_baseline"]
            cb["gpu_over_cpu"] = {"port": value / cb["value"], "early_exit_port": value / cb["early_exit_port"]["value"]}
        print(json.dumps(line), flush=True)
    if dumps is not None:
        np.save(args.dump_gather, torch.stack(dumps).cpu().numpy())
    b.close()
    if distributed:
        dist.destroy_process_group()
    if not checks_ok:
        print(f"bench.py: lane checks failed over the timed window: {bad}", file=sys.stderr, flush=True)
        sys.exit(3)


if __name__ == "__main__":
    main()
