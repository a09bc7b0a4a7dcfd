#!/bin/bash
# Round-4 first GPU session: the GPU suite (new tests: 8-shard composition, cHW repair), the v0
# driver-window bench line with the like-for-like CPU baseline and every diagnostic, and the
# per-phase split (MRP_STAMPS variant library) of every BASELINE config over the same window.
set -uo pipefail
mkdir -p gpurun_out
( for i in $(seq 1 60); do date >> gpurun_out/heartbeat; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4s1_gpu_tests.log 2>&1 \
  || { echo "gpu tests failed"; tail -40 gpurun_out/r4s1_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r4s1_gpu_tests.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r4s1_bench_driver.log 2>&1 \
  || { echo "bench failed"; tail -20 gpurun_out/r4s1_bench_driver.log; exit 1; }
tail -1 gpurun_out/r4s1_bench_driver.log | cut -c1-400
for cfg in "0 4096" "1 4096" "2 1024" "4 1024" "5 4096"; do
  set -- $cfg
  MRP_LIB=gym_puzzles_amd/libmrp_stamps.so timeout -k 10 200 python tools/phase_profile.py $1 $2 5 20 gpurun_out/r4_phase_env$1.json \
      > gpurun_out/r4_phase_env$1.txt 2>&1 || { echo "phase env $1 failed"; tail -20 gpurun_out/r4_phase_env$1.txt; exit 1; }
  head -3 gpurun_out/r4_phase_env$1.txt
done
exit 0
