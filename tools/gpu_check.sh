#!/bin/bash
# One GPU-box session: parity tests (-m gpu), bench, optional phase profiles.
#   tools/gpu_check.sh [envs-to-phase-profile...]
# A heartbeat file under gpurun_out/ keeps a slow first `import torch` from reading as a hang;
# every GPU step still runs under its own timeout and the chain stops at the first failure.
set -uo pipefail
mkdir -p gpurun_out
( for i in $(seq 1 40); do date >> gpurun_out/heartbeat; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
rm -f gpurun_out/phase.txt
for e in "$@"; do
  MRP_LIB=gym_puzzles_amd/libmrp_stamps.so timeout -k 10 120 python tools/phase_profile.py $e 4096 100 >> gpurun_out/phase.txt 2>&1 || { echo "phase profile failed"; tail -20 gpurun_out/phase.txt; exit 1; }
done
exit 0
