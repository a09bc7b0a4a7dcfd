#!/bin/bash
# Round-4 session 18: LLVM's iterative-ilp scheduler (+4.4 % on v0, session 17) on v3 (libmrp_it5,
# with lanes pairs), Heavy-v0 (libmrp_it1, inlined) and the 3-block config (libmrp_it4, loops out of
# line) against the default library: parity, then an interleaved A/B, two rounds.
set -uo pipefail
O=gpurun_out/r4s18
mkdir -p $O
( for i in $(seq 1 80); do date >> gpurun_out/heartbeat; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
T=tests/test_gpu.py
for lib in libmrp_it5:5 libmrp_it1:1 libmrp_it4:4; do
  L=${lib%%:*}; E=${lib##*:}
  MRP_LIB=gym_puzzles_amd/$L.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
      "$T::test_device_autoreset_full_size[$E]" "$T::test_step_parity_host_inputs[$E]" "$T::test_whole_episode_soak[$E]" \
      > $O/tests_$L.log 2>&1 || { echo "gpu tests failed ($L)"; tail -30 $O/tests_$L.log; exit 1; }
  echo "$L parity: $(tail -1 $O/tests_$L.log)"
done
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --later-window 200 --later-start 21 --episode 0 --multi-step 0 --single-env 0"
for round in 1 2; do
  for cfg in 5:4096:libmrp_it5 1:4096:libmrp_it1 4:1024:libmrp_it4; do
    IFS=: read env lanes cand <<< "$cfg"
    for lib in libmrp $cand; do
      MRP_LIB=gym_puzzles_amd/$lib.so timeout -k 10 200 python bench.py --env $env --lanes $lanes $ARGS > $O/ab_${lib}_env${env}_r$round.log 2>&1 \
        || { echo "bench $lib env $env failed"; tail $O/ab_${lib}_env${env}_r$round.log; exit 1; }
      python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; g=d['diagnostics']; print('env', sys.argv[3], sys.argv[2], round(d['value']/1e6,3), 'M/s window; later', round(g['later_window']['env_steps_per_s']/1e6,3), 'kernel_ms', round(d['roofline']['kernel_ms'],4))" \
        $O/ab_${lib}_env${env}_r$round.log $lib $env
    done
  done
done
exit 0
