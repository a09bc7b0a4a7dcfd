"""Lone-wave duration of the launches' slowest lane-steps (diagnostic, GPU box).

    python tools/chain_bench.py OUT.json [--envs 0,2,4] [--repeat 5] [--libs A.so,B.so,...] [--rounds 2]

A launch of k_step lasts as long as its slowest lane-step, one wave's serial solver chain
(DESIGN.md, round 4).  tools/chain_inputs/cap_env<E>.npz hold the pre-step lane states of the
20 slowest lane-steps of bench.py's driver window (steps 6-25 after spawn; captured with
tools/issue_capture.py on the stamps build).  Each is replayed alone as a 1-lane k_step launch
(same seed, global lane and step counter, so the same lane-step bit for bit), `repeat` times, and
timed with HIP events on the launch's stream.  The median per lane-step, their mean and sum go to
OUT.json, with an FNV hash of the lane state after each step: libraries that claim the same bits
must hash the same.  With --libs every library runs in a child process of its own (MRP_LIB), the
libraries interleaved over `rounds` rounds, so variants of the solver compare on one box.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INPUTS = os.path.join(ROOT, "tools", "chain_inputs")


def _fnv(a: np.ndarray) -> str:
    h = 0xcbf29ce484222325
    for w in np.ascontiguousarray(a).view(np.uint64 if a.nbytes % 8 == 0 else np.uint32).tolist():
        h = ((h ^ w) * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
    return f"{h:016x}"


def run_one(envs, repeat):
    import torch
    sys.path.insert(0, ROOT)
    from gym_puzzles_amd import Batch
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(device=dev)
    out = {}
    for env in envs:
        cap = np.load(os.path.join(INPUTS, f"cap_env{env}.npz"))
        rows = []
        for k in range(len(cap["lane"])):
            lane = int(cap["lane"][k])
            b = Batch(env, 1, seed=17, lane_offset=lane)
            b.set_auto_reset(True)
            b.set_stream(s.cuda_stream)
            obs = torch.zeros(b.obs_dim, device=dev)
            rew = torch.zeros(1, device=dev)
            times, h = [], None
            for r in range(repeat + 1):
                b.set_state(cap["state"][k][None])
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                with torch.cuda.stream(s):
                    e0.record(s)
                    b.step_device(None, obs.data_ptr(), rew.data_ptr())
                    e1.record(s)
                s.synchronize()
                if r > 0:   # the first launch of a lane-step warms the code path
                    times.append(e0.elapsed_time(e1) * 1e3)
                hk = _fnv(b.get_state()[0])
                assert h is None or hk == h, f"env {env} row {k}: replay not deterministic"
                h = hk
            b.close()
            rows.append({"row": k, "lane": lane, "us": float(np.median(times)), "us_min": float(np.min(times)), "state_hash": h})
        us = [r["us"] for r in rows]
        out[str(env)] = {"rows": rows, "mean_us": float(np.mean(us)), "sum_us": float(np.sum(us)), "max_us": float(np.max(us))}
        print(f"env {env}: {len(rows)} slowest lane-steps alone: mean {np.mean(us):8.1f} us  max {np.max(us):8.1f} us", flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--envs", default="0,2,4")
    ap.add_argument("--repeat", type=int, default=5)
    ap.add_argument("--libs", default="")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    envs = [int(e) for e in a.envs.split(",")]
    if a.child or not a.libs:
        res = run_one(envs, a.repeat)
        with open(a.out, "w") as f:
            json.dump(res, f)
        return
    libs = a.libs.split(",")
    allres = {lib: [] for lib in libs}
    for rnd in range(a.rounds):
        for lib in libs:
            tmp = a.out + f".{os.path.basename(lib)}.{rnd}.json"
            env = dict(os.environ, MRP_LIB=os.path.abspath(lib))
            print(f"--- round {rnd} {lib}", flush=True)
            subprocess.run([sys.executable, os.path.abspath(__file__), tmp, "--envs", a.envs, "--repeat", str(a.repeat),
                            "--child"], env=env, check=True, timeout=600)
            with open(tmp) as f:
                allres[lib].append(json.load(f))
    summary = {}
    for lib in libs:
        summary[lib] = {e: {"mean_us": [r[str(e)]["mean_us"] for r in allres[lib]],
                            "hashes": [row["state_hash"] for row in allres[lib][0][str(e)]["rows"]]} for e in envs}
    base = libs[0]
    for lib in libs:
        line = []
        for e in envs:
            m = np.mean(summary[lib][e]["mean_us"])
            b0 = np.mean(summary[base][e]["mean_us"])
            same = summary[lib][e]["hashes"] == summary[base][e]["hashes"]
            line.append(f"env {e} {m:8.1f} us ({(b0 / m - 1) * 100:+5.1f} %){'' if same else ' BITS DIFFER'}")
        print(f"{os.path.basename(lib):28s} " + " | ".join(line), flush=True)
    with open(a.out, "w") as f:
        json.dump({"libs": libs, "summary": summary, "runs": allres}, f)


if __name__ == "__main__":
    main()
