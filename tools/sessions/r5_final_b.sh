#!/bin/bash
# Round-5 final evidence, part B (GPU box): issue-roofline capture / replay of the configs whose
# unit changed this round (v0, v2, 3-block; tools/issue_capture.py with the stamps library, replays
# under SQ counters and the kernel trace), merged into profiles/r5_issue_roofline.json on the box,
# the per-phase tables, then the driver-window line of every config with its CPU baselines.
set -uo pipefail
O=gpurun_out/r5fb
mkdir -p $O
( for i in $(seq 1 75); do date >> $O/heartbeat; sleep 15; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
STAMPS=gym_puzzles_amd/libmrp_stamps.so
for cfg in "0 4096" "2 1024" "4 1024"; do
  set -- $cfg
  MRP_LIB=$STAMPS timeout -k 10 200 python tools/issue_capture.py $1 $2 5 20 $O/cap_env$1.npz > $O/cap_env$1.log 2>&1 || { echo "capture $1 failed"; tail $O/cap_env$1.log; exit 1; }
  MRP_LIB=$STAMPS timeout -k 10 200 python tools/issue_replay.py $O/cap_env$1.npz $O/replay_stamps_env$1.json > $O/replay_stamps_env$1.log 2>&1 || { echo "replay $1 failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM SQ_WAVE_CYCLES \
      --output-format csv -d $O/pmc_env$1 -o pmc -- python3 tools/issue_replay.py $O/cap_env$1.npz /tmp/r.json > $O/pmc_env$1.log 2>&1 || { echo "pmc $1 failed"; exit 1; }
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/kt_env$1 -o kt -- python3 tools/issue_replay.py $O/cap_env$1.npz /tmp/r.json 3 \
      > $O/kt_env$1.log 2>&1 || { echo "kt $1 failed"; exit 1; }
  MRP_LIB=$STAMPS timeout -k 10 200 python tools/phase_profile.py $1 $2 5 20 $O/r5_phase_env$1.json > $O/r5_phase_env$1.txt 2>&1 || { echo "phase $1 failed"; exit 1; }
  head -1 $O/r5_phase_env$1.txt
done
python3 tools/issue_roofline.py $O $O/issue_new.json 0 2 4 > $O/issue_roofline.txt || { echo "issue roofline failed"; exit 1; }
python3 -c "import json; a=json.load(open('profiles/r5_issue_roofline.json')); b=json.load(open('$O/issue_new.json')); a={k: v for k, v in a.items() if not k.startswith(('0:', '2:', '4:'))}; a.update(b); json.dump(a, open('profiles/r5_issue_roofline.json', 'w'), indent=1)"
cp profiles/r5_issue_roofline.json $O/
for cfg in "0 4096" "1 4096" "2 1024" "4 1024" "5 4096"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --env $1 --lanes $2 --steps 20 --warmup 5 --later-window 0 --episode 0 --multi-step 0 \
      --single-env 0 > $O/cfg_env$1.log 2>&1 || { echo "bench env $1 failed"; tail -20 $O/cfg_env$1.log; exit 1; }
  tail -1 $O/cfg_env$1.log | cut -c1-160
done
exit 0
