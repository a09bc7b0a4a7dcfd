#!/bin/bash
# Round-6 final evidence, part F (GPU box), after v0 and v3 moved to 4 waves per SIMD (only their units
# changed): the GPU suite and smoke, the driver-window and default bench lines, v0's rocprofv3 set (kernel
# trace + stats, PMC traffic), v3's config line, v0's four windows against round 5, interleaved.
set -uo pipefail
O=gpurun_out/r6ff
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
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || { echo "driver bench failed"; tail -20 $O/bench_driver.log; exit 1; }
tail -1 $O/bench_driver.log | cut -c1-160
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || { echo "default bench failed"; tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log | cut -c1-160
STEPS=20 WARMUP=5 LANES=4096 timeout -k 10 400 bash tools/profile.sh r6_v0 0 > $O/prof_v0.log 2>&1 || { echo "profile 0 failed"; tail $O/prof_v0.log; exit 1; }
tail -1 $O/prof_v0.log | cut -c1-200
timeout -k 10 300 python bench.py --env 5 --lanes 4096 --steps 20 --warmup 5 --later-window 0 --episode 0 --multi-step 0 --single-env 0 \
    > $O/cfg_env5.log 2>&1 || { echo "bench env 5 failed"; tail -20 $O/cfg_env5.log; exit 1; }
tail -1 $O/cfg_env5.log | cut -c1-120
timeout -k 10 700 bash tools/windows_ab.sh r6ff/win "gym_puzzles_amd/var/libmrp_r5.so gym_puzzles_amd/libmrp.so" || { echo "windows failed"; exit 1; }
exit 0
