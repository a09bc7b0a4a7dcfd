#!/bin/bash
# Round-6 final evidence, part B (GPU box): every other BASELINE config's driver-window line with its CPU
# baselines (Heavy-v0, v2, the 3-block config, v3), the Heavy-v0 traffic split, the 2-rank line and the
# RCCL one-rank line; v0's four windows of the round-5 library and the final one; both libraries' slowest lane-steps alone.
set -uo pipefail
O=gpurun_out/r6fb
mkdir -p $O
( for i in $(seq 1 100); do date >> $O/heartbeat; sleep 15; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
for e in 1 2 4 5; do
  L=4096; [ $e = 2 ] && L=1024; [ $e = 4 ] && L=1024
  timeout -k 10 300 python bench.py --env $e --lanes $L --steps 20 --warmup 5 --later-window 0 --episode 0 --multi-step 0 \
      --single-env 0 > $O/cfg_env$e.log 2>&1 || { echo "bench env $e failed"; tail -20 $O/cfg_env$e.log; exit 1; }
  tail -1 $O/cfg_env$e.log | cut -c1-120
done
for e in 0 1; do
  timeout -k 10 200 python tools/traffic_split.py $e 4096 5 20 $O/traffic_split_env$e.json > $O/traffic_split_env$e.txt 2>&1 \
    || { echo "traffic split $e failed"; tail $O/traffic_split_env$e.txt; exit 1; }
  tail -1 $O/traffic_split_env$e.txt
done
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29561 bench.py \
    --gpus 2 --dist-backend gloo --same-device --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_2rank.log 2>&1 \
  || { echo "2-rank bench failed"; tail -20 $O/bench_2rank.log; exit 1; }
grep '"metric"' $O/bench_2rank.log | cut -c1-200
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port 29562 bench.py \
    --gpus 1 --dist-backend nccl --force-collective --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_rccl1.log 2>&1 \
  || { echo "rccl bench failed"; tail -20 $O/bench_rccl1.log; exit 1; }
grep '"metric"' $O/bench_rccl1.log | cut -c1-200
timeout -k 10 700 bash tools/windows_ab.sh r6fb/win "gym_puzzles_amd/var/libmrp_r5.so gym_puzzles_amd/libmrp.so" \
  || { echo "windows failed"; exit 1; }
timeout -k 10 600 python -u tools/chain_bench.py $O/chain.json --envs 0,1,2,4,5 --repeat 3 --rounds 2 \
  --libs gym_puzzles_amd/var/libmrp_r5.so,gym_puzzles_amd/libmrp.so > $O/chain.log 2>&1 \
  || { echo "chain bench failed"; tail -20 $O/chain.log; exit 1; }
tail -2 $O/chain.log
exit 0
