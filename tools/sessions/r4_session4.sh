#!/bin/bash
# Round-4 session 4 (new default build): the GPU suite; late-dispatched lanes' priority A/B
# (MRP_LATE_PRIO 0..3, envs 0 and 5, interleaved); lane-index phase split with the priority on;
# instruction-cache counters of the v0 driver window.
set -uo pipefail
O=gpurun_out/r4s4
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
  for env in 0 5; do
    for lp in 0 1 2 3; do
      MRP_LATE_PRIO=$lp timeout -k 10 200 python bench.py --env $env $ARGS > $O/ab_lp${lp}_env${env}_r$round.log 2>&1 \
        || { echo "bench lp$lp env$env failed"; tail $O/ab_lp${lp}_env${env}_r$round.log; exit 1; }
      python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; g=d['diagnostics']; print('env', sys.argv[3], 'late_prio', sys.argv[2], round(d['value']/1e6,3), 'M/s window; later', round(g['later_window']['env_steps_per_s']/1e6,3), 'episode', round(g['whole_episode']['env_steps_per_s']/1e6,3), 'kernel_ms', round(d['roofline']['kernel_ms'],4))" $O/ab_lp${lp}_env${env}_r$round.log $lp $env
    done
  done
done
for lp in 0 2; do
  MRP_LATE_PRIO=$lp MRP_LIB=gym_puzzles_amd/libmrp_stamps.so timeout -k 10 200 python tools/lane_phases.py 0 4096 5 20 $O/lanes_lp${lp}_env0.json > $O/lanes_lp${lp}_env0.txt 2>&1 \
    || { echo "lane phases failed"; tail $O/lanes_lp${lp}_env0.txt; exit 1; }
  echo "late_prio $lp"; cat $O/lanes_lp${lp}_env0.txt
done
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS \
    --output-format csv -d $O/icache -o icache -- python3 bench.py $ARGS --episode 0 --later-window 0 > $O/icache.log 2>&1 \
  || { echo "icache pmc failed"; tail $O/icache.log; exit 1; }
python3 tools/pmc_summary.py $O/icache k_step > $O/icache_summary.txt 2>&1; cat $O/icache_summary.txt
exit 0
