#!/bin/bash
# GPU tests on a candidate library, velbench on it, then the interleaved bench A/B of several builds
#   tools/ab3.sh <candidate.so> <other.so>...
set -uo pipefail
CAND=$1
mkdir -p gpurun_out
( for i in $(seq 1 80); do date >> gpurun_out/heartbeat; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
MRP_LIB=$CAND timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_gpu_tests.log 2>&1 \
  || { echo "gpu tests failed"; tail -40 gpurun_out/ab_gpu_tests.log; exit 1; }
tail -1 gpurun_out/ab_gpu_tests.log
MRP_LIB=$CAND timeout -k 10 120 python tools/velbench.py > gpurun_out/velbench_cand.txt 2>&1 || { echo "velbench failed"; exit 1; }
grep "blocks     1" gpurun_out/velbench_cand.txt
timeout -k 10 900 bash tools/ab_bench.sh "$@" $CAND || exit 1
