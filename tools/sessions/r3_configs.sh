#!/bin/bash
# Per-config GPU + CPU numbers for BASELINE.md (GPU box): the driver-window bench line (steps 6-25,
# CPU baseline on the allotted cores and 1 lane / 1 core) for every BASELINE config at its per-GPU
# lane count, then the rocprofv3 profile of v0 over the same window (kernel trace, HBM traffic,
# VALU instruction counters).  The chain stops at the first failure.
set -uo pipefail
TAG=${1:-r3b}
mkdir -p gpurun_out
( for i in $(seq 1 60); do date >> gpurun_out/heartbeat; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
for cfg in "0 4096" "1 4096" "2 1024" "4 1024" "5 4096"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --env $1 --lanes $2 --steps 20 --warmup 5 --later-window 0 --episode 0 --multi-step 0 \
      --single-env 0 > gpurun_out/cfg_env$1.log 2>&1 || { echo "bench env $1 failed"; tail -20 gpurun_out/cfg_env$1.log; exit 1; }
  tail -1 gpurun_out/cfg_env$1.log | cut -c1-400
done
STEPS=20 WARMUP=5 LANES=4096 VALU_PMC=1 timeout -k 10 600 bash tools/profile.sh ${TAG}_v0_drv 0 || { echo "profile failed"; exit 1; }
exit 0
