#!/bin/bash
# Round-4 session 7: late-dispatched lanes raise their issue priority before their state load
# (mrp_lane.h k_step, MRP_LATE_PRIO=k).  Parity of the new build (env 0/1/5, with and without the
# raised priority), then an interleaved A/B of the driver window on the configs that have late lanes
# (v0, Heavy-v0, v3 at 4096 lanes) against the previous build, and the load marks of each lane block.
set -uo pipefail
O=gpurun_out/r4s7
mkdir -p $O
( for i in $(seq 1 80); do date >> gpurun_out/heartbeat; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
T=tests/test_gpu.py
for P in 0 3; do
  MRP_LATE_PRIO=$P timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
      "$T::test_device_autoreset_full_size[0]" "$T::test_device_autoreset_full_size[1]" "$T::test_device_autoreset_full_size[5]" \
      "$T::test_step_parity_host_inputs[0]" "$T::test_step_parity_host_inputs[5]" > $O/tests_p$P.log 2>&1 \
    || { echo "gpu tests failed (late prio $P)"; tail -30 $O/tests_p$P.log; exit 1; }
  echo "late prio $P: $(tail -1 $O/tests_p$P.log)"
done
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --later-window 200 --later-start 21 --episode 0 --multi-step 0 --single-env 0"
for round in 1 2; do
  for env in 0 1 5; do
    for v in old:0 new:0 new:2 new:3; do
      lib=${v%%:*}; P=${v##*:}
      so=gym_puzzles_amd/libmrp.so; [ $lib = old ] && so=gym_puzzles_amd/libmrp_old.so
      MRP_LIB=$so MRP_LATE_PRIO=$P timeout -k 10 200 python bench.py --env $env $ARGS > $O/ab_${lib}_p${P}_env${env}_r$round.log 2>&1 \
        || { echo "bench $v env $env failed"; tail $O/ab_${lib}_p${P}_env${env}_r$round.log; exit 1; }
      python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; g=d['diagnostics']; print('env', sys.argv[3], sys.argv[2], round(d['value']/1e6,3), 'M/s window; later', round(g['later_window']['env_steps_per_s']/1e6,3), 'kernel_ms', round(d['roofline']['kernel_ms'],4))" \
        $O/ab_${lib}_p${P}_env${env}_r$round.log $v $env
    done
  done
done
for env in 0 5; do
  for P in 0 3; do
    MRP_LIB=gym_puzzles_amd/libmrp_stamps.so MRP_LATE_PRIO=$P timeout -k 10 200 python tools/lane_phases.py $env 4096 5 20 $O/lanes_env${env}_p$P.json \
        > $O/lanes_env${env}_p$P.txt 2>&1 || { echo "lane_phases env $env failed"; tail $O/lanes_env${env}_p$P.txt; exit 1; }
    echo "== env $env late prio $P"; cat $O/lanes_env${env}_p$P.txt
  done
done
exit 0
