#!/bin/bash
# Round-4 session 14: the narrow phase of up to 32 contacts on groups of 8 / 4 / 2 lanes per contact
# (libmrp_cg: -DMRP_COLLIDE_GROUPS=1, envs 0 2 5) against the default library: parity, then an
# interleaved A/B of v2, v0 and v3 in the driver window, three rounds.
set -uo pipefail
O=gpurun_out/r4s14
mkdir -p $O
( for i in $(seq 1 80); do date >> gpurun_out/heartbeat; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
T=tests/test_gpu.py
MRP_LIB=gym_puzzles_amd/libmrp_cg.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    "$T::test_device_autoreset_full_size[0]" "$T::test_device_autoreset_full_size[2]" "$T::test_device_autoreset_full_size[5]" \
    "$T::test_whole_episode_soak[2]" "$T::test_step_parity_host_inputs[0]" "$T::test_step_parity_host_inputs[2]" "$T::test_whole_episode_soak[0]" "$T::test_device_autoreset_full_size[1]" > $O/tests_gr.log 2>&1 \
  || { echo "gpu tests failed (collide groups)"; tail -30 $O/tests_gr.log; exit 1; }
echo "collide groups parity: $(tail -1 $O/tests_gr.log)"
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --later-window 200 --later-start 21 --episode 0 --multi-step 0 --single-env 0"
for round in 1 2 3; do
  for cfg in 2:1024 0:4096 5:4096; do
    env=${cfg%%:*}; lanes=${cfg##*:}
    for lib in libmrp libmrp_cg; do
      MRP_LIB=gym_puzzles_amd/$lib.so timeout -k 10 200 python bench.py --env $env --lanes $lanes $ARGS > $O/ab_${lib}_env${env}_r$round.log 2>&1 \
        || { echo "bench $lib env $env failed"; tail $O/ab_${lib}_env${env}_r$round.log; exit 1; }
      python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; g=d['diagnostics']; print('env', sys.argv[3], sys.argv[2], round(d['value']/1e6,3), 'M/s window; later', round(g['later_window']['env_steps_per_s']/1e6,3), 'kernel_ms', round(d['roofline']['kernel_ms'],4))" \
        $O/ab_${lib}_env${env}_r$round.log $lib $env
    done
  done
done
exit 0
