#!/bin/bash
# Round-6 session 4 (GPU box): libmrp_r6c.so (ONE_ROT rotations evaluated only for contacts with a rotating
# body, the pass snapshot in LDS, the redo through rot(); cooperative fixture synchronisation) - GPU
# suite, slowest lane-steps against r6b, posbench, phase tables (var/stamps_r6c.so), traffic split.
set -uo pipefail
O=gpurun_out/r6s4
mkdir -p $O
( for i in $(seq 1 100); do date >> $O/heartbeat; sleep 15; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
MRP_LIB=gym_puzzles_amd/libmrp_r6c.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  || { echo "gpu tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
MRP_LIB=gym_puzzles_amd/libmrp_r6c.so timeout -k 10 120 python -u tools/posbench.py > $O/posbench_r6c.txt 2>&1 \
  || { echo "posbench failed"; tail $O/posbench_r6c.txt; exit 1; }
grep "blocks     1" $O/posbench_r6c.txt
timeout -k 10 600 python -u tools/chain_bench.py $O/chain.json --envs 0,1,2,4,5 --repeat 3 --rounds 2 \
  --libs gym_puzzles_amd/libmrp_r6b.so,gym_puzzles_amd/libmrp_r6c.so > $O/chain.log 2>&1 \
  || { echo "chain bench failed"; tail -20 $O/chain.log; exit 1; }
tail -2 $O/chain.log
for e in 0 1 2 4 5; do
  L=4096; [ $e = 2 ] && L=1024; [ $e = 4 ] && L=1024
  MRP_LIB=gym_puzzles_amd/var/stamps_r6c.so timeout -k 10 200 python tools/phase_profile.py $e $L 5 20 $O/phase_env$e.json > $O/phase_env$e.txt 2>&1 \
    || { echo "phase $e failed"; tail $O/phase_env$e.txt; exit 1; }
  head -24 $O/phase_env$e.txt
done
for e in 0 1; do
  MRP_LIB=gym_puzzles_amd/libmrp_r6c.so timeout -k 10 200 python tools/traffic_split.py $e 4096 5 20 $O/traffic_split_env$e.json > $O/traffic_split_env$e.txt 2>&1 \
    || { echo "traffic split $e failed"; tail $O/traffic_split_env$e.txt; exit 1; }
  cat $O/traffic_split_env$e.txt
done
exit 0
