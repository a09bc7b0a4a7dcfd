#!/bin/bash
# Round-3 GPU-box check: parity tests (-m gpu), the driver-window bench line (with the CPU
# baseline, as the driver runs it), the default bench line, and a kernel-trace profile of the
# driver window (its per-launch k_step average over exactly the timed launches).  Each GPU step
# has its own time limit; the chain stops at the first failure.
#   tools/sessions/r3_session.sh <tag> [skip-tests]
set -uo pipefail
TAG=${1:-r3}
mkdir -p gpurun_out
( for i in $(seq 1 60); do date >> gpurun_out/heartbeat; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 \
    || { echo "gpu tests failed"; tail -40 gpurun_out/gpu_tests_$TAG.log; exit 1; }
  tail -1 gpurun_out/gpu_tests_$TAG.log
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_driver_$TAG.log 2>&1 \
  || { echo "bench (driver window) failed"; tail -20 gpurun_out/bench_driver_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_driver_$TAG.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_default_$TAG.log 2>&1 \
  || { echo "bench (default) failed"; tail -20 gpurun_out/bench_default_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_default_$TAG.log
OUT=gpurun_out/prof_${TAG}_drv
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 bench.py --steps 20 --warmup 5 \
  --no-cpu-baseline --later-window 0 --episode 0 --multi-step 0 --single-env 0 > $OUT/kt.log 2>&1 \
  || { echo "rocprof failed"; tail -20 $OUT/kt.log; exit 1; }
python3 tools/kt_window.py "$(find $OUT/kt -name '*kernel_trace.csv' -print -quit)" 5 20 $OUT/kt.log
exit 0
