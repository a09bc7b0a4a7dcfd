#!/bin/bash
# Round-4 session 8: the sparse early-exit schedule (compare every 4 sweeps up to sweep 32, then
# every 16; libmrp_exit.so, envs 0 1 2 4 5) against the current library: parity first, then an
# interleaved A/B of every config's driver window; then the entry probes of the stamps build
# (instruction fetch of 1 KB of cold code, first load of the lane state) by lane block.
set -uo pipefail
O=gpurun_out/r4s8
mkdir -p $O
( for i in $(seq 1 80); do date >> gpurun_out/heartbeat; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
T=tests/test_gpu.py
MRP_LIB=gym_puzzles_amd/libmrp_exit.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    "$T::test_device_autoreset_full_size[0]" "$T::test_device_autoreset_full_size[1]" "$T::test_device_autoreset_full_size[2]" \
    "$T::test_device_autoreset_full_size[4]" "$T::test_device_autoreset_full_size[5]" \
    "$T::test_step_parity_host_inputs[0]" "$T::test_step_parity_host_inputs[2]" "$T::test_step_parity_host_inputs[4]" \
    "$T::test_whole_episode_soak[0]" "$T::test_whole_episode_soak[4]" > $O/tests_exit.log 2>&1 \
  || { echo "gpu tests failed (exit schedule)"; tail -30 $O/tests_exit.log; exit 1; }
echo "exit schedule parity: $(tail -1 $O/tests_exit.log)"
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --later-window 200 --later-start 21 --episode 0 --multi-step 0 --single-env 0"
for round in 1 2; do
  for cfg in 0:4096 1:4096 2:1024 4:1024 5:4096; do
    env=${cfg%%:*}; lanes=${cfg##*:}
    for lib in libmrp libmrp_exit; do
      MRP_LIB=gym_puzzles_amd/$lib.so timeout -k 10 200 python bench.py --env $env --lanes $lanes $ARGS > $O/ab_${lib}_env${env}_r$round.log 2>&1 \
        || { echo "bench $lib env $env failed"; tail $O/ab_${lib}_env${env}_r$round.log; exit 1; }
      python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; g=d['diagnostics']; print('env', sys.argv[3], sys.argv[2], round(d['value']/1e6,3), 'M/s window; later', round(g['later_window']['env_steps_per_s']/1e6,3), 'kernel_ms', round(d['roofline']['kernel_ms'],4))" \
        $O/ab_${lib}_env${env}_r$round.log $lib $env
    done
  done
done
MRP_LIB=gym_puzzles_amd/libmrp_stamps.so timeout -k 10 200 python tools/lane_phases.py 0 4096 5 20 $O/lanes_env0_probes.json \
    > $O/lanes_env0_probes.txt 2>&1 || { echo "lane_phases failed"; tail $O/lanes_env0_probes.txt; exit 1; }
cat $O/lanes_env0_probes.txt
exit 0
