#!/bin/bash
# Round-4 session 5: the k_step with one env-step call site (code 1.05 -> 0.54 MB for v0): GPU suite,
# interleaved A/B against the previous library (libmrp_old.so) on every BASELINE config, icache
# counters of both, lane-index phase split with the load sub-stamps.
set -uo pipefail
O=gpurun_out/r4s5
mkdir -p $O
( for i in $(seq 1 80); do date >> gpurun_out/heartbeat; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  || { echo "gpu tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --later-window 200 --later-start 21 --episode 1 --multi-step 0 --single-env 0"
for round in 1 2; do
  for cfg in "0 4096" "1 4096" "2 1024" "4 1024" "5 4096"; do
    set -- $cfg
    for lib in libmrp_old libmrp; do
      MRP_LIB=gym_puzzles_amd/$lib.so timeout -k 10 200 python bench.py --env $1 --lanes $2 $ARGS > $O/ab_${lib}_env$1_r$round.log 2>&1 \
        || { echo "bench $lib env$1 failed"; tail $O/ab_${lib}_env$1_r$round.log; exit 1; }
      python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; g=d['diagnostics']; print('env', sys.argv[3], sys.argv[2], round(d['value']/1e6,3), 'M/s window; later', round(g['later_window']['env_steps_per_s']/1e6,3), 'episode', round(g['whole_episode']['env_steps_per_s']/1e6,3), 'kernel_ms', round(d['roofline']['kernel_ms'],4))" $O/ab_${lib}_env$1_r$round.log $lib $1
    done
  done
done
for lib in libmrp_old libmrp; do
  MRP_LIB=gym_puzzles_amd/$lib.so timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS \
      --output-format csv -d $O/icache_$lib -o icache -- python3 bench.py --env 0 --steps 20 --warmup 5 --no-cpu-baseline --later-window 0 --episode 0 --multi-step 0 --single-env 0 > $O/icache_$lib.log 2>&1 \
    || { echo "icache pmc failed"; tail $O/icache_$lib.log; exit 1; }
  echo $lib; python3 tools/pmc_summary.py $O/icache_$lib k_step
done
MRP_LIB=gym_puzzles_amd/libmrp_stamps.so timeout -k 10 200 python tools/lane_phases.py 0 4096 5 20 $O/lanes_env0.json > $O/lanes_env0.txt 2>&1 \
  || { echo "lane phases failed"; tail $O/lanes_env0.txt; exit 1; }
cat $O/lanes_env0.txt
for cfg in "0 4096" "1 4096" "2 1024" "4 1024" "5 4096"; do
  set -- $cfg
  MRP_LIB=gym_puzzles_amd/libmrp_stamps.so timeout -k 10 200 python tools/phase_profile.py $1 $2 5 20 $O/phase_env$1.json > $O/phase_env$1.txt 2>&1 \
      || { echo "phase env $1 failed"; tail -20 $O/phase_env$1.txt; exit 1; }
  head -1 $O/phase_env$1.txt
done
exit 0
