"""BASELINE.md's per-config table from the committed per-config bench lines (CPU only).

    python tools/baseline_table.py profiles/r4f_configs_driver_window.jsonl

Each line is bench.py's JSON for one BASELINE config in the driver window (steps 6-25), with its
like-for-like CPU baseline and roofline objects; prints one markdown row per config."""
import json
import sys

NAMES = {0: "MultiRobotPuzzle-v0 (configs[1])", 1: "MultiRobotPuzzleHeavy-v0 (configs[2])",
         2: "MultiRobotPuzzle-v2 (configs[3], 8192 over 8 GPUs)", 4: "MultiRobotPuzzleHeavy-v2 3-block (configs[4], 8192 over 8 GPUs)",
         5: "MultiRobotPuzzle-v3 (§8f-4)"}


def m(x):
    return f"{x / 1e6:.2f} M" if x >= 1e6 else f"{x / 1e3:.0f} K"


def main():
    rows = [json.loads(l) for l in open(sys.argv[1]) if l.strip()]
    print("| config | lanes/GPU | GPU env-steps/s | `k_step` ms | HBM GB/s (frac) | PMC traffic / launch | issue floor ms (frac) "
          "| slowest lane-step alone, ms | CPU port, 16 cores (window) | early-exit port, 16 cores | CPU 1 lane / 1 core "
          "| GPU ÷ port | GPU ÷ early-exit port |")
    print("|" + "---|" * 13)
    for d in rows:
        env = d["config"]["env_id"]
        r, cb = d["roofline"], d["cpu_baseline"]
        iss = r.get("issue") or {}
        tr = r.get("traffic")
        print(f"| {NAMES.get(env, env)} | {d['config']['lanes_per_gpu']} | **{m(d['value'])}** | {r['kernel_ms']:.3f} "
              f"| {r['achieved']:.1f} ({r['frac']:.4f}) | {tr / 1e6:.1f} MB | "
              + (f"{iss['floor_ms']:.3f} ({iss['frac']:.2f})" if iss else "—") + " | "
              + (f"{iss['lone_wave_ms']:.3f}" if iss else "—")
              + f" | {m(cb['value'])} | {m(cb['early_exit_port']['value'])} | {m(cb['single_lane_1core']['value'])} "
              f"| {d['value'] / cb['value']:.2f} | {d['value'] / cb['early_exit_port']['value']:.2f} |")


if __name__ == "__main__":
    main()
