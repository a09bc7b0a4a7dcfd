#!/bin/bash
# One GPU-box A/B session: parity tests on the current libmrp.so, then velbench and the
# bench windows for each library given:  tools/ab_session.sh libA.so libB.so ...
set -uo pipefail
mkdir -p gpurun_out
( for i in $(seq 1 60); do date >> gpurun_out/heartbeat; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for lib in "$@"; do
  echo "== velbench $lib" | tee -a gpurun_out/velbench.txt
  MRP_LIB=$lib timeout -k 10 120 python tools/velbench.py >> gpurun_out/velbench.txt 2>&1 || { echo "velbench failed"; tail gpurun_out/velbench.txt; exit 1; }
done
cat gpurun_out/velbench.txt
timeout -k 10 900 bash tools/ab_bench.sh "$@" || exit 1
