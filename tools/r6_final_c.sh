#!/bin/bash
# Round-6 final evidence, part C (GPU box): issue roofline recaptured on the final library for v0, Heavy-v0
# and v2 (slowest lane-step of every driver-window launch captured with the stamps build, replayed alone
# under SQ counters and the kernel trace) and the phase tables of envs 0, 1, 2, 4, 5.
set -uo pipefail
O=gpurun_out/r6fc
mkdir -p $O
( for i in $(seq 1 100); do date >> $O/heartbeat; sleep 15; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
STAMPS=gym_puzzles_amd/var/stamps_final3.so
for e in 0 1 2; do
  L=4096; [ $e = 2 ] && L=1024
  MRP_LIB=$STAMPS timeout -k 10 200 python tools/issue_capture.py $e $L 5 20 $O/cap_env$e.npz > $O/cap_env$e.log 2>&1 || { echo "capture failed"; tail $O/cap_env$e.log; exit 1; }
  MRP_LIB=$STAMPS timeout -k 10 200 python tools/issue_replay.py $O/cap_env$e.npz $O/replay_stamps_env$e.json > $O/replay_stamps_env$e.log 2>&1 || { echo "replay failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM SQ_WAVE_CYCLES \
      --output-format csv -d $O/pmc_env$e -o pmc -- python3 tools/issue_replay.py $O/cap_env$e.npz /tmp/r.json > $O/pmc_env$e.log 2>&1 || { echo "pmc failed"; exit 1; }
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/kt_env$e -o kt -- python3 tools/issue_replay.py $O/cap_env$e.npz /tmp/r.json 3 \
      > $O/kt_env$e.log 2>&1 || { echo "kt failed"; exit 1; }
done
python3 tools/issue_roofline.py $O $O/issue_new.json 0 1 2 > $O/issue_roofline.txt || { echo "issue roofline failed"; exit 1; }
cat $O/issue_roofline.txt | head -30
for e in 0 1 2 4 5; do
  L=4096; [ $e = 2 ] && L=1024; [ $e = 4 ] && L=1024
  MRP_LIB=$STAMPS timeout -k 10 200 python tools/phase_profile.py $e $L 5 20 $O/phase_env$e.json > $O/phase_env$e.txt 2>&1 \
    || { echo "phase $e failed"; tail $O/phase_env$e.txt; exit 1; }
  head -1 $O/phase_env$e.txt
done
exit 0
