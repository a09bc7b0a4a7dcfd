#!/bin/bash
# Round-6 session 5 (GPU box): the ONE_ROT passes with the rotation chosen per point (per-contact flag) (libmrp_wt3.so: envs 0
# and 1 from the working tree, the rest r6c) - GPU suite, posbench, slowest lane-steps against the
# default library (r6c + v0 without PICK2_VT), v0 / Heavy-v0 phase tables (var/stamps_wt3.so).
set -uo pipefail
O=gpurun_out/r6s5b
mkdir -p $O
( for i in $(seq 1 80); do date >> $O/heartbeat; sleep 15; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
MRP_LIB=gym_puzzles_amd/libmrp_wt3.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  || { echo "gpu tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
MRP_LIB=gym_puzzles_amd/libmrp_wt3.so timeout -k 10 120 python -u tools/posbench.py > $O/posbench_wt3.txt 2>&1 \
  || { echo "posbench failed"; tail $O/posbench_wt3.txt; exit 1; }
grep "blocks     1" $O/posbench_wt3.txt
timeout -k 10 600 python -u tools/chain_bench.py $O/chain.json --envs 0,1 --repeat 3 --rounds 2 \
  --libs gym_puzzles_amd/libmrp.so,gym_puzzles_amd/libmrp_wt3.so > $O/chain.log 2>&1 \
  || { echo "chain bench failed"; tail -20 $O/chain.log; exit 1; }
tail -2 $O/chain.log
for e in 0 1; do
  MRP_LIB=gym_puzzles_amd/var/stamps_wt3.so timeout -k 10 200 python tools/phase_profile.py $e 4096 5 20 $O/phase_env$e.json > $O/phase_env$e.txt 2>&1 \
    || { echo "phase $e failed"; tail $O/phase_env$e.txt; exit 1; }
  head -24 $O/phase_env$e.txt
done
exit 0
