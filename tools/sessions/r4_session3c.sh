#!/bin/bash
# Round-4 session 3c: parity of the two-body register paths (libmrp_xw.so, env 0) on the env-0 GPU
# tests, then an interleaved driver-window A/B: base library vs xw, and xw with the lane state in
# one contiguous allocation (MRP_STATE_ALLOC=contiguous).
set -uo pipefail
O=gpurun_out/r4s3c
mkdir -p $O
( for i in $(seq 1 60); do date >> gpurun_out/heartbeat; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
T="tests/test_gpu.py::test_step_parity_host_inputs[0] tests/test_gpu.py::test_golden_trajectory[0] tests/test_gpu.py::test_reference_test_flow_v0_seed17 tests/test_gpu.py::test_device_autoreset_full_size[0] tests/test_gpu.py::test_whole_episode_soak[0] tests/test_gpu.py::test_multi_step_launch_equals_single_steps[0] tests/test_gpu.py::test_frameskip_parity[0-2] tests/test_gpu.py::test_nonfinite_lane_is_flagged_not_fatal[0]"
MRP_LIB=gym_puzzles_amd/libmrp_xw.so timeout -k 10 400 python -u -m pytest $T -x -q --timeout 300 --timeout-method thread > $O/xw_tests.log 2>&1 \
  || { echo "xw tests failed"; tail -30 $O/xw_tests.log; exit 1; }
tail -1 $O/xw_tests.log
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --later-window 200 --later-start 21 --episode 1 --multi-step 0 --single-env 0"
for round in 1 2; do
  for v in base xw xwc; do
    case $v in base) LIB=libmrp; EXTRA="";; xw) LIB=libmrp_xw; EXTRA="";; xwc) LIB=libmrp_xw; EXTRA="MRP_STATE_ALLOC=contiguous";; esac
    env $EXTRA MRP_LIB=gym_puzzles_amd/$LIB.so timeout -k 10 200 python bench.py --env 0 $ARGS > $O/ab_${v}_r$round.log 2>&1 \
      || { echo "bench $v failed"; tail $O/ab_${v}_r$round.log; exit 1; }
    python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; g=d['diagnostics']; print(sys.argv[2], round(d['value']/1e6,3), 'M/s window; later', round(g['later_window']['env_steps_per_s']/1e6,3), 'episode', round(g['whole_episode']['env_steps_per_s']/1e6,3), 'kernel_ms', round(d['roofline']['kernel_ms'],4))" $O/ab_${v}_r$round.log $v
  done
done
exit 0
