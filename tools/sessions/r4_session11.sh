#!/bin/bash
# Round-4 session 11: register-path sweeps in pairs (libmrp_pair.so = batched load + sparse exit + paired
# sweeps, envs 0 1 2 4 5) against libmrp_bl.so: whole GPU suite on the candidate, then an interleaved
# A/B of every config (costliest-first dispatch as a third arm).
set -uo pipefail
O=gpurun_out/r4s11
mkdir -p $O
( for i in $(seq 1 80); do date >> gpurun_out/heartbeat; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
MRP_LIB=gym_puzzles_amd/libmrp_pair.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    > $O/tests_pair.log 2>&1 || { echo "gpu suite failed (paired sweeps)"; tail -30 $O/tests_pair.log; exit 1; }
echo "paired sweeps, GPU suite: $(tail -1 $O/tests_pair.log)"
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --later-window 200 --later-start 21 --episode 0 --multi-step 0 --single-env 0"
for round in 1 2; do
  for cfg in 0:4096 1:4096 2:1024 4:1024 5:4096; do
    env=${cfg%%:*}; lanes=${cfg##*:}
    for arm in libmrp_bl:0 libmrp_pair:0 libmrp_pair:1; do
      lib=${arm%%:*}; s=${arm##*:}
      MRP_LIB=gym_puzzles_amd/$lib.so timeout -k 10 200 python bench.py --env $env --lanes $lanes --schedule $s $ARGS > $O/ab_${lib}_s${s}_env${env}_r$round.log 2>&1 \
        || { echo "bench $arm env $env failed"; tail $O/ab_${lib}_s${s}_env${env}_r$round.log; exit 1; }
      python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; g=d['diagnostics']; print('env', sys.argv[3], sys.argv[2], round(d['value']/1e6,3), 'M/s window; later', round(g['later_window']['env_steps_per_s']/1e6,3), 'kernel_ms', round(d['roofline']['kernel_ms'],4))" \
        $O/ab_${lib}_s${s}_env${env}_r$round.log $arm $env
    done
  done
done
exit 0
