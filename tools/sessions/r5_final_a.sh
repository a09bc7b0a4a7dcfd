#!/bin/bash
# Round-5 final evidence, part A (GPU box): the GPU suite, smoke, the v0 rocprofv3 set (kernel
# trace + stats, FETCH_SIZE, WRITE_SIZE, VALU counters -> profiles/), then the driver-window and
# default bench lines and the 2-rank (gloo, one device) bench line.  Stops at the first failure.
set -uo pipefail
O=gpurun_out/r5fa
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
STEPS=20 WARMUP=5 LANES=4096 VALU_PMC=1 timeout -k 10 400 bash tools/profile.sh r5_v0 0 > /dev/null || { echo "profile 0 failed"; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || { echo "driver bench failed"; tail -20 $O/bench_driver.log; exit 1; }
tail -1 $O/bench_driver.log | cut -c1-200
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || { echo "default bench failed"; tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log | cut -c1-160
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29561 bench.py \
    --gpus 2 --dist-backend gloo --same-device --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_2rank.log 2>&1 \
  || { echo "2-rank bench failed"; tail -20 $O/bench_2rank.log; exit 1; }
grep '"metric"' $O/bench_2rank.log | cut -c1-200
exit 0
