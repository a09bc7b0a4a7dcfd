#!/bin/bash
# Round-6 session 7b (GPU box): session 7 (tools/r6_s7.sh), then the issue roofline of the 3-block config
# and v3 recaptured on the final library (as tools/r6_final_c.sh does for v0, Heavy-v0 and v2).
set -uo pipefail
bash tools/r6_s7.sh || exit 1
O=gpurun_out/r6s7b
mkdir -p $O
( for i in $(seq 1 60); do date >> $O/heartbeat; sleep 15; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
STAMPS=gym_puzzles_amd/var/stamps_final3.so
for e in 4 5; do
  L=4096; [ $e = 4 ] && L=1024
  MRP_LIB=$STAMPS timeout -k 10 200 python tools/issue_capture.py $e $L 5 20 $O/cap_env$e.npz > $O/cap_env$e.log 2>&1 || { echo "capture failed"; tail $O/cap_env$e.log; exit 1; }
  MRP_LIB=$STAMPS timeout -k 10 200 python tools/issue_replay.py $O/cap_env$e.npz $O/replay_stamps_env$e.json > $O/replay_stamps_env$e.log 2>&1 || { echo "replay failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM SQ_WAVE_CYCLES \
      --output-format csv -d $O/pmc_env$e -o pmc -- python3 tools/issue_replay.py $O/cap_env$e.npz /tmp/r.json > $O/pmc_env$e.log 2>&1 || { echo "pmc failed"; exit 1; }
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/kt_env$e -o kt -- python3 tools/issue_replay.py $O/cap_env$e.npz /tmp/r.json 3 \
      > $O/kt_env$e.log 2>&1 || { echo "kt failed"; exit 1; }
done
python3 tools/issue_roofline.py $O $O/issue_new.json 4 5 > $O/issue_roofline.txt || { echo "issue roofline failed"; exit 1; }
grep "^env" $O/issue_roofline.txt
exit 0
