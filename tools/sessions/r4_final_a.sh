#!/bin/bash
# Round-4 final evidence, first call: the GPU suite, smoke, the driver-window bench line of every
# BASELINE config with its like-for-like CPU baseline (oracle port and early-exit port on the GPU
# line's window, whole episode, 1 lane / 1 core), then the default and driver-window v0 lines with
# every diagnostic.  The chain stops at the first failure.
set -uo pipefail
O=gpurun_out/r4f
mkdir -p $O
( for i in $(seq 1 75); do date >> gpurun_out/heartbeat; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  || { echo "gpu tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
  || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for cfg in "0 4096" "1 4096" "2 1024" "4 1024" "5 4096"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --env $1 --lanes $2 --steps 20 --warmup 5 --later-window 0 --episode 0 --multi-step 0 \
      --single-env 0 > $O/cfg_env$1.log 2>&1 || { echo "bench env $1 failed"; tail -20 $O/cfg_env$1.log; exit 1; }
  tail -1 $O/cfg_env$1.log | cut -c1-200
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || { echo "driver bench failed"; tail -20 $O/bench_driver.log; exit 1; }
tail -1 $O/bench_driver.log | cut -c1-300
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || { echo "default bench failed"; tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log | cut -c1-200
exit 0
