#!/bin/bash
# Round-6 final evidence, part A (GPU box): the GPU suite and smoke on the default library, the v0
# rocprofv3 set (kernel trace + stats, FETCH_SIZE, WRITE_SIZE, VALU counters -> profiles/), the
# Heavy-v0 PMC traffic, the driver-window and default bench lines.  Stops at the first failure.
set -uo pipefail
O=gpurun_out/r6fa
mkdir -p $O
( for i in $(seq 1 100); do date >> $O/heartbeat; sleep 15; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  || { echo "gpu tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
  || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
STEPS=20 WARMUP=5 LANES=4096 VALU_PMC=1 timeout -k 10 400 bash tools/profile.sh r6_v0 0 > $O/prof_v0.log 2>&1 || { echo "profile 0 failed"; tail $O/prof_v0.log; exit 1; }
tail -3 $O/prof_v0.log
STEPS=20 WARMUP=5 LANES=4096 timeout -k 10 400 bash tools/profile.sh r6_heavy_v0 1 > $O/prof_v1.log 2>&1 || { echo "profile 1 failed"; tail $O/prof_v1.log; exit 1; }
tail -3 $O/prof_v1.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || { echo "driver bench failed"; tail -20 $O/bench_driver.log; exit 1; }
tail -1 $O/bench_driver.log | cut -c1-200
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || { echo "default bench failed"; tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log | cut -c1-160
exit 0
