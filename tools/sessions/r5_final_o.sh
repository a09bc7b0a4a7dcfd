#!/bin/bash
# Round-5 final evidence after v0 took the lanes-path branch-free selection: the GPU suite, smoke,
# the v0 rocprofv3 set, v0's issue roofline / phase table (var/stamps0b.so), v0's driver-window
# config line with CPU baselines, the driver-window and default bench lines and the 2-rank line.
set -uo pipefail
O=gpurun_out/r5fo
mkdir -p $O
( for i in $(seq 1 75); do date >> $O/heartbeat; sleep 15; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  || { echo "gpu tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
  || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
STEPS=20 WARMUP=5 LANES=4096 VALU_PMC=1 timeout -k 10 400 bash tools/profile.sh r5e_v0 0 > /dev/null || { echo "profile 0 failed"; exit 1; }
STAMPS=gym_puzzles_amd/var/stamps0b.so
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
tail -1 $O/cfg_env0.log | cut -c1-120
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || { echo "driver bench failed"; tail -20 $O/bench_driver.log; exit 1; }
tail -1 $O/bench_driver.log | cut -c1-200
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || { echo "default bench failed"; tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log | cut -c1-160
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29561 bench.py \
    --gpus 2 --dist-backend gloo --same-device --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_2rank.log 2>&1 \
  || { echo "2-rank bench failed"; tail -20 $O/bench_2rank.log; exit 1; }
grep '"metric"' $O/bench_2rank.log | cut -c1-200
exit 0
