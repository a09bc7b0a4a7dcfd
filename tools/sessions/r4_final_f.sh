#!/bin/bash
# Round-4 final evidence after v2 took the max-ilp scheduler (only the env-2 unit changed): the
# GPU suite, smoke, v2's rocprofv3 set (kernel trace + stats, FETCH_SIZE, WRITE_SIZE) and its
# issue-roofline capture / replay (merged into profiles/r4_issue_roofline.json on the box), then
# the driver-window line of every config with its CPU baselines and the driver-window / default
# v0 lines.  The chain stops at the first failure.
set -uo pipefail
O=gpurun_out/r4ff
O2=gpurun_out/r4ff2
mkdir -p $O $O2
( for i in $(seq 1 75); do date >> gpurun_out/heartbeat; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  || { echo "gpu tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
  || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
STEPS=20 WARMUP=5 LANES=1024 timeout -k 10 400 bash tools/profile.sh r4j_v2 2 > /dev/null || { echo "profile 2 failed"; exit 1; }
STAMPS=gym_puzzles_amd/libmrp_stamps.so
MRP_LIB=$STAMPS timeout -k 10 200 python tools/issue_capture.py 2 1024 5 20 $O2/cap_env2.npz > $O2/cap_env2.log 2>&1 || { echo "capture failed"; exit 1; }
MRP_LIB=$STAMPS timeout -k 10 200 python tools/issue_replay.py $O2/cap_env2.npz $O2/replay_stamps_env2.json > $O2/replay_stamps_env2.log 2>&1 || { echo "replay failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM SQ_WAVE_CYCLES \
    --output-format csv -d $O2/pmc_env2 -o pmc -- python3 tools/issue_replay.py $O2/cap_env2.npz /tmp/r.json > $O2/pmc_env2.log 2>&1 || { echo "pmc failed"; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O2/kt_env2 -o kt -- python3 tools/issue_replay.py $O2/cap_env2.npz /tmp/r.json 3 \
    > $O2/kt_env2.log 2>&1 || { echo "kt failed"; exit 1; }
MRP_LIB=$STAMPS timeout -k 10 200 python tools/phase_profile.py 2 1024 5 20 $O2/r4_phase_env2.json > $O2/r4_phase_env2.txt 2>&1 || { echo "phase failed"; exit 1; }
python3 tools/issue_roofline.py $O2 $O2/issue_env2.json 2 > $O2/issue_roofline.txt || { echo "issue roofline failed"; exit 1; }
python3 -c "import json; a=json.load(open('profiles/r4_issue_roofline.json')); b=json.load(open('$O2/issue_env2.json')); a={k: v for k, v in a.items() if not k.startswith('2:')}; a.update(b); json.dump(a, open('profiles/r4_issue_roofline.json', 'w'), indent=1)"
cp profiles/r4_issue_roofline.json $O2/
for cfg in "0 4096" "1 4096" "2 1024" "4 1024" "5 4096"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --env $1 --lanes $2 --steps 20 --warmup 5 --later-window 0 --episode 0 --multi-step 0 \
      --single-env 0 > $O/cfg_env$1.log 2>&1 || { echo "bench env $1 failed"; tail -20 $O/cfg_env$1.log; exit 1; }
  tail -1 $O/cfg_env$1.log | cut -c1-160
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || { echo "driver bench failed"; tail -20 $O/bench_driver.log; exit 1; }
tail -1 $O/bench_driver.log | cut -c1-200
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || { echo "default bench failed"; tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log | cut -c1-160
exit 0
