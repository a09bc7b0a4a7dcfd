"""Average duration of the k_step launches of bench.py's timed window, from a rocprofv3 kernel
trace (the --kernel-trace CSV), so the profile's figure covers exactly the launches bench.py's
HIP events time: the first `warmup` k_step launches are skipped and the next `steps` are averaged
(run bench.py with the diagnostics off so no other k_step launch follows the window).

    python tools/kt_window.py <kernel_trace.csv> <warmup> <steps> [bench.json] > window.json
"""
from __future__ import annotations

import csv
import json
import sys


def window(path: str, warmup: int, steps: int) -> dict:
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            if "k_step" in name:
                rows.append((int(r["Dispatch_Id"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    if len(rows) < warmup + steps:
        raise SystemExit(f"{path}: {len(rows)} k_step launches, fewer than warmup {warmup} + steps {steps}")
    win = rows[warmup:warmup + steps]
    durs = [(e - s) * 1e-6 for _, s, e, _ in win]    # ns -> ms
    span = (win[-1][2] - win[0][1]) * 1e-6
    return {"kernel": win[0][3], "launches_in_trace": len(rows), "skipped_warmup": warmup, "window_launches": steps,
            "mean_ms": sum(durs) / steps, "min_ms": min(durs), "max_ms": max(durs),
            "first_start_to_last_end_ms_per_launch": span / steps}


if __name__ == "__main__":
    out = window(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]))
    if len(sys.argv) > 4:
        with open(sys.argv[4]) as f:
            line = next(json.loads(x) for x in f if x.startswith("{") and '"metric"' in x)
        out["bench_kernel_ms"] = line["roofline"]["kernel_ms"]
        out["bench_ms_per_step"] = line["ms_per_step"]
        out["bench_kernel_ms_timing"] = line["roofline"]["kernel_ms_timing"]
    print(json.dumps(out))
