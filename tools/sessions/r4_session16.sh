#!/bin/bash
# Round-4 session 16: the max-ilp machine scheduler on the inlined k_step of v0 / v3
# (libmrp_ilp05: -DMRP_LANES_PAIRS=1 + max-ilp, envs 0 5) and v2 (libmrp_ilp2: granules + max-ilp,
# env 2) against the default library (Heavy-v0 gained 6.5 % from it, profiles/r4_ab_unit_flags.txt):
# parity, then an interleaved A/B of the driver window, three rounds.
set -uo pipefail
O=gpurun_out/r4s16
mkdir -p $O
( for i in $(seq 1 80); do date >> gpurun_out/heartbeat; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
T=tests/test_gpu.py
MRP_LIB=gym_puzzles_amd/libmrp_ilp05.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    "$T::test_device_autoreset_full_size[0]" "$T::test_device_autoreset_full_size[5]" "$T::test_step_parity_host_inputs[0]" \
    "$T::test_whole_episode_soak[0]" > $O/tests_ilp05.log 2>&1 || { echo "gpu tests failed (ilp05)"; tail -30 $O/tests_ilp05.log; exit 1; }
MRP_LIB=gym_puzzles_amd/libmrp_ilp2.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    "$T::test_device_autoreset_full_size[2]" "$T::test_step_parity_host_inputs[2]" "$T::test_whole_episode_soak[2]" \
    > $O/tests_ilp2.log 2>&1 || { echo "gpu tests failed (ilp2)"; tail -30 $O/tests_ilp2.log; exit 1; }
echo "parity: $(tail -1 $O/tests_ilp05.log) / $(tail -1 $O/tests_ilp2.log)"
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --later-window 200 --later-start 21 --episode 0 --multi-step 0 --single-env 0"
for round in 1 2 3; do
  for cfg in 0:4096:libmrp_ilp05 2:1024:libmrp_ilp2 5:4096:libmrp_ilp05; do
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
