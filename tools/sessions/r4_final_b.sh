#!/bin/bash
# Round-4 final evidence, second call: the rocprofv3 set of every BASELINE config over the driver
# window (kernel trace + stats, FETCH_SIZE, WRITE_SIZE in separate passes; tools/profile.sh), then
# the issue-count roofline inputs (tools/sessions/r4_session2.sh's capture / replay with the atomic-free
# stamps build): the launches' slowest lane-steps captured in the batch, replayed alone under the
# SQ_INSTS counters and the kernel trace.  Local half: tools/collect_profiles.sh r4f and
# tools/issue_roofline.py gpurun_out/r4f2 profiles/r4_issue_roofline.json.
set -uo pipefail
O=gpurun_out/r4f2
mkdir -p $O
( for i in $(seq 1 75); do date >> gpurun_out/heartbeat; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
STEPS=20 WARMUP=5 LANES=4096 VALU_PMC=1 timeout -k 10 400 bash tools/profile.sh r4f_v0 0 > /dev/null || { echo "profile v0 failed"; exit 1; }
STEPS=20 WARMUP=5 LANES=4096 timeout -k 10 400 bash tools/profile.sh r4f_heavy_v0 1 > /dev/null || { echo "profile 1 failed"; exit 1; }
STEPS=20 WARMUP=5 LANES=1024 timeout -k 10 400 bash tools/profile.sh r4f_v2 2 > /dev/null || { echo "profile 2 failed"; exit 1; }
STEPS=20 WARMUP=5 LANES=1024 timeout -k 10 400 bash tools/profile.sh r4f_heavy_v2_3block 4 > /dev/null || { echo "profile 4 failed"; exit 1; }
STEPS=20 WARMUP=5 LANES=4096 timeout -k 10 400 bash tools/profile.sh r4f_v3 5 > /dev/null || { echo "profile 5 failed"; exit 1; }
mkdir -p $O/profiles && cp profiles/pmc_traffic.json profiles/r4f_* $O/profiles/
echo "profiles done"
STAMPS=gym_puzzles_amd/libmrp_stamps.so
for cfg in "0 4096" "1 4096" "2 1024" "4 1024" "5 4096"; do
  set -- $cfg
  MRP_LIB=$STAMPS timeout -k 10 200 python tools/issue_capture.py $1 $2 5 20 $O/cap_env$1.npz > $O/cap_env$1.log 2>&1 \
    || { echo "capture $1 failed"; tail $O/cap_env$1.log; exit 1; }
  MRP_LIB=$STAMPS timeout -k 10 200 python tools/issue_replay.py $O/cap_env$1.npz $O/replay_stamps_env$1.json > $O/replay_stamps_env$1.log 2>&1 \
    || { echo "stamps replay $1 failed"; tail $O/replay_stamps_env$1.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM SQ_WAVE_CYCLES \
      --output-format csv -d $O/pmc_env$1 -o pmc -- python3 tools/issue_replay.py $O/cap_env$1.npz /tmp/r.json > $O/pmc_env$1.log 2>&1 \
    || { echo "pmc $1 failed"; tail $O/pmc_env$1.log; exit 1; }
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/kt_env$1 -o kt -- python3 tools/issue_replay.py $O/cap_env$1.npz /tmp/r.json 3 \
      > $O/kt_env$1.log 2>&1 || { echo "kt $1 failed"; tail $O/kt_env$1.log; exit 1; }
  MRP_LIB=$STAMPS timeout -k 10 200 python tools/phase_profile.py $1 $2 5 20 $O/r4_phase_env$1.json > $O/r4_phase_env$1.txt 2>&1 \
    || { echo "phase $1 failed"; tail $O/r4_phase_env$1.txt; exit 1; }
  echo "env $1 captured"
done
timeout -k 10 200 python tools/single_env_timing.py MultiRobotPuzzle-v0 300 > $O/single_env.log 2>&1 || { echo "single env failed"; tail $O/single_env.log; exit 1; }
cat $O/single_env.log
exit 0
