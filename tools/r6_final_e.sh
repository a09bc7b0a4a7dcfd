#!/bin/bash
# Round-6 final evidence, part E (GPU box), after v3 took BFREE_LANES (only the v3 unit changed): the GPU
# suite and smoke on the final library, the driver-window and default bench lines, v3's config line with
# its CPU baselines, v3's rocprofv3 set (kernel trace + stats, PMC traffic), and v3's later window and whole
# episode against the previous library (var/libmrp_final3.so), interleaved.
set -uo pipefail
O=gpurun_out/r6fe
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
timeout -k 10 300 python bench.py --env 5 --lanes 4096 --steps 20 --warmup 5 --later-window 0 --episode 0 --multi-step 0 --single-env 0 \
    > $O/cfg_env5.log 2>&1 || { echo "bench env 5 failed"; tail -20 $O/cfg_env5.log; exit 1; }
tail -1 $O/cfg_env5.log | cut -c1-120
STEPS=20 WARMUP=5 LANES=4096 timeout -k 10 400 bash tools/profile.sh r6_v3 5 > $O/prof_v3.log 2>&1 || { echo "profile 5 failed"; tail $O/prof_v3.log; exit 1; }
tail -2 $O/prof_v3.log | cut -c1-200
for r in 0 1; do
  for lib in gym_puzzles_amd/var/libmrp_final3.so gym_puzzles_amd/libmrp.so; do
    n=$(basename $lib .so)
    MRP_LIB=$lib timeout -k 10 300 python bench.py --env 5 --steps 200 --warmup 20 --no-cpu-baseline --single-env 0 --later-window 200 --episode 1 --multi-step 0 \
        > $O/v3win_${n}_$r.log 2>&1 || { echo "v3 windows failed"; tail -20 $O/v3win_${n}_$r.log; exit 1; }
    python3 - $O/v3win_${n}_$r.log $n $r <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
g = d["diagnostics"]
print(f"round {sys.argv[3]} {sys.argv[2]:18s} steps 21-220 {d['value'] / 1e6:7.3f} M  later window {g['later_window']['env_steps_per_s'] / 1e6:7.3f} M  whole episode {g['whole_episode']['env_steps_per_s'] / 1e6:7.3f} M")
PY
  done
done
exit 0
