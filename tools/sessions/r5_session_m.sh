#!/bin/bash
# Round 5: Heavy-v0 / v3 with the two-ballot case test and the cross-product tangent speed
# (var/pv15.so) against the default library (slowest lane-steps alone), then v0's issue roofline and
# phase table recaptured on the final library (var/stamps24.so: the stamps build of the v0 unit) and
# v0's driver-window line with its CPU baselines.
set -uo pipefail
O=gpurun_out/r5sm
mkdir -p $O
( for i in $(seq 1 75); do date >> $O/heartbeat; sleep 15; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
STAMPS=gym_puzzles_amd/var/stamps24.so
for e in 2 4; do
  MRP_LIB=$STAMPS timeout -k 10 200 python tools/issue_capture.py $e 1024 5 20 $O/cap_env$e.npz > $O/cap_env$e.log 2>&1 || { echo "capture failed"; tail $O/cap_env$e.log; exit 1; }
  MRP_LIB=$STAMPS timeout -k 10 200 python tools/issue_replay.py $O/cap_env$e.npz $O/replay_stamps_env$e.json > $O/replay_stamps_env$e.log 2>&1 || { echo "replay failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM SQ_WAVE_CYCLES \
      --output-format csv -d $O/pmc_env$e -o pmc -- python3 tools/issue_replay.py $O/cap_env$e.npz /tmp/r.json > $O/pmc_env$e.log 2>&1 || { echo "pmc failed"; exit 1; }
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/kt_env$e -o kt -- python3 tools/issue_replay.py $O/cap_env$e.npz /tmp/r.json 3 \
      > $O/kt_env$e.log 2>&1 || { echo "kt failed"; exit 1; }
  MRP_LIB=$STAMPS timeout -k 10 200 python tools/phase_profile.py $e 1024 5 20 $O/r5_phase_env$e.json > $O/r5_phase_env$e.txt 2>&1 || { echo "phase failed"; exit 1; }
  head -1 $O/r5_phase_env$e.txt
done
python3 tools/issue_roofline.py $O $O/issue_new.json 2 4 > $O/issue_roofline.txt || { echo "issue roofline failed"; exit 1; }
python3 -c "import json; a=json.load(open('profiles/r5_issue_roofline.json')); b=json.load(open('$O/issue_new.json')); a={k: v for k, v in a.items() if not k.startswith(('2:', '4:'))}; a.update(b); json.dump(a, open('profiles/r5_issue_roofline.json', 'w'), indent=1)"
cp profiles/r5_issue_roofline.json $O/
exit 0
