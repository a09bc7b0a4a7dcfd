#!/bin/bash
# Round-3 final evidence on the GPU box, one call: the GPU suite, smoke, the driver-window bench
# line of every BASELINE config (CPU port on the allotted cores + 1 lane / 1 core beside it), the
# rocprofv3 set of every config over the same window (kernel trace, FETCH_SIZE, WRITE_SIZE; VALU
# counters for v0), then the default and driver-window v0 lines with every diagnostic.
# Local half: WARMUP=5 STEPS=20 tools/collect_profiles.sh <tag>.  The chain stops at the first failure.
#   tools/sessions/r3_final.sh [tag]   (default r3f)
set -uo pipefail
TAG=${1:-r3f}
mkdir -p gpurun_out
( for i in $(seq 1 75); do date >> gpurun_out/heartbeat; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final_gpu_tests.log 2>&1 \
  || { echo "gpu tests failed"; tail -30 gpurun_out/final_gpu_tests.log; exit 1; }
tail -1 gpurun_out/final_gpu_tests.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1 \
  || { echo "smoke failed"; tail -20 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
for cfg in "0 4096" "1 4096" "2 1024" "4 1024" "5 4096"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --env $1 --lanes $2 --steps 20 --warmup 5 --later-window 0 --episode 0 --multi-step 0 \
      --single-env 0 > gpurun_out/final_cfg_env$1.log 2>&1 || { echo "bench env $1 failed"; tail -20 gpurun_out/final_cfg_env$1.log; exit 1; }
  tail -1 gpurun_out/final_cfg_env$1.log | cut -c1-300
done
STEPS=20 WARMUP=5 LANES=4096 VALU_PMC=1 timeout -k 10 400 bash tools/profile.sh ${TAG}_v0 0 > /dev/null || { echo "profile v0 failed"; exit 1; }
STEPS=20 WARMUP=5 LANES=4096 timeout -k 10 400 bash tools/profile.sh ${TAG}_heavy_v0 1 > /dev/null || { echo "profile 1 failed"; exit 1; }
STEPS=20 WARMUP=5 LANES=1024 timeout -k 10 400 bash tools/profile.sh ${TAG}_v2 2 > /dev/null || { echo "profile 2 failed"; exit 1; }
STEPS=20 WARMUP=5 LANES=1024 timeout -k 10 400 bash tools/profile.sh ${TAG}_heavy_v2_3block 4 > /dev/null || { echo "profile 4 failed"; exit 1; }
STEPS=20 WARMUP=5 LANES=4096 timeout -k 10 400 bash tools/profile.sh ${TAG}_v3 5 > /dev/null || { echo "profile 5 failed"; exit 1; }
echo "profiles done"
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || { echo "default bench failed"; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2>&1 || { echo "driver bench failed"; exit 1; }
tail -1 gpurun_out/bench_driver.log | cut -c1-300
exit 0
