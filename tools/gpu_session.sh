#!/bin/bash
# One GPU-box check: parity tests (-m gpu), the driver-window bench, the default bench, and a
# slow-lane replay on the stamps build.  Each GPU step has its own time limit; the chain stops at
# the first failure.
set -uo pipefail
mkdir -p gpurun_out
( for i in $(seq 1 40); do date >> gpurun_out/heartbeat; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_drv.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_drv.log; exit 1; }
tail -1 gpurun_out/bench_drv.log
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bench_def.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_def.log; exit 1; }
tail -1 gpurun_out/bench_def.log
if [ -f gym_puzzles_amd/libmrp_stamps.so ]; then
  MRP_LIB=gym_puzzles_amd/libmrp_stamps.so timeout -k 10 120 python tools/lane_replay.py 0 4096 8 5 > gpurun_out/replay.txt 2>&1 || { echo "replay failed"; tail gpurun_out/replay.txt; exit 1; }
  cat gpurun_out/replay.txt
fi
if [ -f gym_puzzles_amd/libmrp_stamps.so ]; then
  MRP_LIB=gym_puzzles_amd/libmrp_stamps.so timeout -k 10 200 python tools/contention.py 0 4096 8 > gpurun_out/contention.txt 2>&1 || { echo "contention failed"; tail gpurun_out/contention.txt; exit 1; }
  cat gpurun_out/contention.txt
fi
