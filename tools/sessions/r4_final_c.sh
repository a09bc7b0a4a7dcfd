#!/bin/bash
# Round-4 final evidence on the final library (contact slots moved word by word): the GPU suite,
# smoke, the rocprofv3 set of every BASELINE config (kernel trace + stats, FETCH_SIZE, WRITE_SIZE;
# tools/profile.sh writes profiles/pmc_traffic.json on the box), then the driver-window bench line
# of every config -- which reads that fresh traffic table and the committed issue roofline -- with
# its like-for-like CPU baseline, the driver-window and default v0 lines with every diagnostic,
# and the v3 TOI-event split of the stamps build.  The chain stops at the first failure.
set -uo pipefail
O=gpurun_out/r4fc
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
STEPS=20 WARMUP=5 LANES=4096 VALU_PMC=1 timeout -k 10 400 bash tools/profile.sh r4g_v0 0 > /dev/null || { echo "profile v0 failed"; exit 1; }
STEPS=20 WARMUP=5 LANES=4096 timeout -k 10 400 bash tools/profile.sh r4g_heavy_v0 1 > /dev/null || { echo "profile 1 failed"; exit 1; }
STEPS=20 WARMUP=5 LANES=1024 timeout -k 10 400 bash tools/profile.sh r4g_v2 2 > /dev/null || { echo "profile 2 failed"; exit 1; }
STEPS=20 WARMUP=5 LANES=1024 timeout -k 10 400 bash tools/profile.sh r4g_heavy_v2_3block 4 > /dev/null || { echo "profile 4 failed"; exit 1; }
STEPS=20 WARMUP=5 LANES=4096 timeout -k 10 400 bash tools/profile.sh r4g_v3 5 > /dev/null || { echo "profile 5 failed"; exit 1; }
echo "profiles done"
for cfg in "0 4096" "1 4096" "2 1024" "4 1024" "5 4096"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --env $1 --lanes $2 --steps 20 --warmup 5 --later-window 0 --episode 0 --multi-step 0 \
      --single-env 0 > $O/cfg_env$1.log 2>&1 || { echo "bench env $1 failed"; tail -20 $O/cfg_env$1.log; exit 1; }
  tail -1 $O/cfg_env$1.log | cut -c1-160
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || { echo "driver bench failed"; tail -20 $O/bench_driver.log; exit 1; }
tail -1 $O/bench_driver.log | cut -c1-200
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || { echo "default bench failed"; tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log | cut -c1-160
MRP_LIB=gym_puzzles_amd/libmrp_stamps.so timeout -k 10 200 python tools/phase_profile.py 5 4096 5 20 $O/phase_env5_events.json \
    > $O/phase_env5_events.txt 2>&1 || { echo "phase env 5 failed"; tail $O/phase_env5_events.txt; exit 1; }
cat $O/phase_env5_events.txt
exit 0
