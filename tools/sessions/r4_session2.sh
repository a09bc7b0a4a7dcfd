#!/bin/bash
# Round-4 second GPU session: the lane-steps that set each launch's duration, captured in the
# driver window (stamps library) and replayed alone -- phase split alone (stamps), executed
# instruction counts (rocprofv3 SQ_INSTS_* counters) and lone-wave durations (kernel trace) --
# for every BASELINE config; the load-phase scaling of v0 with the lane count; the single-env split.
set -uo pipefail
mkdir -p gpurun_out/r4s2
( for i in $(seq 1 80); do date >> gpurun_out/heartbeat; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
O=gpurun_out/r4s2
STAMPS=gym_puzzles_amd/libmrp_stamps.so
for cfg in "0 4096" "1 4096" "2 1024" "4 1024" "5 4096"; do
  set -- $cfg
  MRP_LIB=$STAMPS timeout -k 10 200 python tools/issue_capture.py $1 $2 5 20 $O/cap_env$1.npz > $O/cap_env$1.log 2>&1 \
    || { echo "capture $1 failed"; tail $O/cap_env$1.log; exit 1; }
  tail -1 $O/cap_env$1.log
  MRP_LIB=$STAMPS timeout -k 10 200 python tools/issue_replay.py $O/cap_env$1.npz $O/replay_stamps_env$1.json > $O/replay_stamps_env$1.log 2>&1 \
    || { echo "stamps replay $1 failed"; tail $O/replay_stamps_env$1.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM SQ_WAVE_CYCLES \
      --output-format csv -d $O/pmc_env$1 -o pmc -- python3 tools/issue_replay.py $O/cap_env$1.npz /tmp/r.json > $O/pmc_env$1.log 2>&1 \
    || { echo "pmc $1 failed"; tail $O/pmc_env$1.log; exit 1; }
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/kt_env$1 -o kt -- python3 tools/issue_replay.py $O/cap_env$1.npz /tmp/r.json 3 \
      > $O/kt_env$1.log 2>&1 || { echo "kt $1 failed"; tail $O/kt_env$1.log; exit 1; }
done
echo "replays done"
for L in 256 1024 2048; do
  MRP_LIB=$STAMPS timeout -k 10 200 python tools/phase_profile.py 0 $L 5 20 $O/phase_env0_L$L.json > $O/phase_env0_L$L.txt 2>&1 \
    || { echo "phase L$L failed"; exit 1; }
  sed -n 1,4p $O/phase_env0_L$L.txt; grep store $O/phase_env0_L$L.txt
done
timeout -k 10 200 python tools/single_env_timing.py MultiRobotPuzzle-v0 300 > $O/single_env.log 2>&1 || { echo "single env failed"; tail $O/single_env.log; exit 1; }
cat $O/single_env.log
exit 0
