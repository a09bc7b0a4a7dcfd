#!/bin/bash
# A/B session on the GPU box: GPU parity tests on the candidate library (gym_puzzles_amd/libmrp.so),
# the velocity micro-benchmark on both libraries, then the interleaved bench A/B.
#   tools/ab_session.sh <base.so> [skip-tests]
set -uo pipefail
BASE=${1:-gym_puzzles_amd/libmrp_base.so}
mkdir -p gpurun_out
( for i in $(seq 1 60); do date >> gpurun_out/heartbeat; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_gpu_tests.log 2>&1 \
    || { echo "gpu tests failed"; tail -40 gpurun_out/ab_gpu_tests.log; exit 1; }
  tail -1 gpurun_out/ab_gpu_tests.log
fi
for lib in $BASE gym_puzzles_amd/libmrp.so; do
  echo "== velbench $lib"
  MRP_LIB=$lib timeout -k 10 120 python tools/velbench.py > gpurun_out/velbench_$(basename $lib .so).txt 2>&1 || { echo "velbench failed"; exit 1; }
  grep "blocks     1" gpurun_out/velbench_$(basename $lib .so).txt
done
timeout -k 10 600 bash tools/ab_bench.sh $BASE gym_puzzles_amd/libmrp.so || exit 1
exit 0
