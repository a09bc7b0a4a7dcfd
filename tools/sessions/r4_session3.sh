#!/bin/bash
# Round-4 session 3: occupancy A/B (3 vs 4 waves per SIMD for k_step, envs 0 and 5) in the driver
# window, interleaved, and the per-lane phase split by lane-index block for both occupancies.
set -uo pipefail
O=gpurun_out/r4s3
mkdir -p $O
( for i in $(seq 1 60); do date >> gpurun_out/heartbeat; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --later-window 200 --later-start 21 --episode 0 --multi-step 0 --single-env 0"
for round in 1 2; do
  for env in 0 5; do
    for lib in libmrp libmrp_w4; do
      MRP_LIB=gym_puzzles_amd/$lib.so timeout -k 10 120 python bench.py --env $env $ARGS > $O/ab_${lib}_env${env}_r$round.log 2>&1 \
        || { echo "bench $lib $env failed"; tail $O/ab_${lib}_env${env}_r$round.log; exit 1; }
      python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[2], sys.argv[3], round(d['value']/1e6,3), 'M/s window; later', round(d['diagnostics']['later_window']['env_steps_per_s']/1e6,3), 'kernel_ms', round(d['roofline']['kernel_ms'],4))" $O/ab_${lib}_env${env}_r$round.log $lib $env
    done
  done
done
for env in 0 5; do
  for lib in libmrp_stamps libmrp_w4_stamps; do
    MRP_LIB=gym_puzzles_amd/$lib.so timeout -k 10 200 python tools/lane_phases.py $env 4096 5 20 $O/lanes_${lib}_env$env.json > $O/lanes_${lib}_env$env.txt 2>&1 \
      || { echo "lane phases $lib $env failed"; tail $O/lanes_${lib}_env$env.txt; exit 1; }
    echo "$lib env $env"; cat $O/lanes_${lib}_env$env.txt
  done
done
exit 0
