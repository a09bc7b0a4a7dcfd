#!/bin/bash
# Round 5: Heavy-v0 / v3 with the two-ballot case test and the cross-product tangent speed
# (var/pv15.so) against the default library (slowest lane-steps alone), then v0's issue roofline and
# phase table recaptured on the final library (var/stamps0.so: the stamps build of the v0 unit) and
# v0's driver-window line with its CPU baselines.
set -uo pipefail
O=gpurun_out/r5se
mkdir -p $O
( for i in $(seq 1 75); do date >> $O/heartbeat; sleep 15; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/chain_bench.py $O/chain.json --envs 1,5 --repeat 5 --rounds 2 \
    --libs gym_puzzles_amd/libmrp.so,gym_puzzles_amd/var/pv15.so > $O/chain.txt 2>&1 || { echo "chain failed"; tail $O/chain.txt; exit 1; }
tail -3 $O/chain.txt
STAMPS=gym_puzzles_amd/var/stamps0.so
MRP_LIB=$STAMPS timeout -k 10 200 python tools/issue_capture.py 0 4096 5 20 $O/cap_env0.npz > $O/cap_env0.log 2>&1 || { echo "capture failed"; tail $O/cap_env0.log; exit 1; }
MRP_LIB=$STAMPS timeout -k 10 200 python tools/issue_replay.py $O/cap_env0.npz $O/replay_stamps_env0.json > $O/replay_stamps_env0.log 2>&1 || { echo "replay failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM SQ_WAVE_CYCLES \
    --output-format csv -d $O/pmc_env0 -o pmc -- python3 tools/issue_replay.py $O/cap_env0.npz /tmp/r.json > $O/pmc_env0.log 2>&1 || { echo "pmc failed"; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/kt_env0 -o kt -- python3 tools/issue_replay.py $O/cap_env0.npz /tmp/r.json 3 \
    > $O/kt_env0.log 2>&1 || { echo "kt failed"; exit 1; }
MRP_LIB=$STAMPS timeout -k 10 200 python tools/phase_profile.py 0 4096 5 20 $O/r5_phase_env0.json > $O/r5_phase_env0.txt 2>&1 || { echo "phase failed"; exit 1; }
head -1 $O/r5_phase_env0.txt
python3 tools/issue_roofline.py $O $O/issue_new.json 0 > $O/issue_roofline.txt || { echo "issue roofline failed"; exit 1; }
python3 -c "import json; a=json.load(open('profiles/r5_issue_roofline.json')); b=json.load(open('$O/issue_new.json')); a={k: v for k, v in a.items() if not k.startswith('0:')}; a.update(b); json.dump(a, open('profiles/r5_issue_roofline.json', 'w'), indent=1)"
cp profiles/r5_issue_roofline.json $O/
timeout -k 10 300 python bench.py --env 0 --lanes 4096 --steps 20 --warmup 5 --later-window 0 --episode 0 --multi-step 0 \
    --single-env 0 > $O/cfg_env0.log 2>&1 || { echo "bench env 0 failed"; tail -20 $O/cfg_env0.log; exit 1; }
tail -1 $O/cfg_env0.log | cut -c1-160
exit 0
