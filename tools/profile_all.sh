#!/bin/bash
# Round profile set (GPU box): rocprofv3 kernel stats + HBM traffic for the BASELINE configs at
# their per-GPU lane counts, then the default bench line (with the CPU baseline).
#   tools/profile_all.sh <round-tag>
set -uo pipefail
R=$1
mkdir -p gpurun_out profiles
( for i in $(seq 1 60); do date >> gpurun_out/heartbeat; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
LANES=4096 timeout -k 10 400 bash tools/profile.sh ${R}_v0 0 || exit 1
LANES=4096 timeout -k 10 400 bash tools/profile.sh ${R}_heavy_v0 1 || exit 1
LANES=1024 timeout -k 10 400 bash tools/profile.sh ${R}_v2 2 || exit 1
LANES=1024 timeout -k 10 400 bash tools/profile.sh ${R}_heavy_v2_3block 4 || exit 1
LANES=4096 timeout -k 10 400 bash tools/profile.sh ${R}_v3 5 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || exit 1
grep -h '"metric"' gpurun_out/bench_default.log > profiles/${R}_bench_default.json
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_driver.log 2>&1 || exit 1
grep -h '"metric"' gpurun_out/bench_driver.log > profiles/${R}_bench_driver_window.json
exit 0
