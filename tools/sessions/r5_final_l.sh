#!/bin/bash
# Round-5 final evidence after v2 / 3-block took MRP_VEL_BFREE=2: the GPU suite, smoke, the v2 and
# 3-block rocprofv3 sets, their driver-window config lines with CPU baselines, then the v0
# driver-window and default bench lines and the 2-rank line.  Stops at the first failure.
set -uo pipefail
O=gpurun_out/r5fl
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
STEPS=20 WARMUP=5 LANES=1024 timeout -k 10 400 bash tools/profile.sh r5d_v2 2 > /dev/null || { echo "profile 2 failed"; exit 1; }
STEPS=20 WARMUP=5 LANES=1024 timeout -k 10 400 bash tools/profile.sh r5d_heavy_v2_3block 4 > /dev/null || { echo "profile 4 failed"; exit 1; }
for e in 2 4; do
  timeout -k 10 300 python bench.py --env $e --lanes 1024 --steps 20 --warmup 5 --later-window 0 --episode 0 --multi-step 0 \
      --single-env 0 > $O/cfg_env$e.log 2>&1 || { echo "bench env $e failed"; tail -20 $O/cfg_env$e.log; exit 1; }
  tail -1 $O/cfg_env$e.log | cut -c1-120
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || { echo "driver bench failed"; tail -20 $O/bench_driver.log; exit 1; }
tail -1 $O/bench_driver.log | cut -c1-200
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || { echo "default bench failed"; tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log | cut -c1-160
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29561 bench.py \
    --gpus 2 --dist-backend gloo --same-device --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_2rank.log 2>&1 \
  || { echo "2-rank bench failed"; tail -20 $O/bench_2rank.log; exit 1; }
grep '"metric"' $O/bench_2rank.log | cut -c1-200
exit 0
