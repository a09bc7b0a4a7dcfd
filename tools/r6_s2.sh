#!/bin/bash
# Round-6 session 2 (GPU box): the rebuilt library (ONE_ROT position passes, TOI far-pair skip, dropped
# arms removed) against the round-5 library (var/libmrp_r5.so):
#  - the GPU suite on the new library (bitwise vs the oracle, incl. the block-angle range test)
#  - posbench, new vs round 5
#  - the launches' slowest lane-steps replayed alone (chain_bench: envs 0, 1, 2, 4, 5), both libraries
#  - v0 bench windows (driver, steps 21-220, 501-700, whole episode): round 5, its PICK2_VT / BFREE_LANES
#    A/B builds, the new library
set -uo pipefail
O=gpurun_out/r6s2
mkdir -p $O
( for i in $(seq 1 160); do date >> $O/heartbeat; sleep 15; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  || { echo "gpu tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for lib in var/libmrp_r5 libmrp; do
  n=$(basename $lib)
  MRP_LIB=gym_puzzles_amd/$lib.so timeout -k 10 120 python -u tools/posbench.py > $O/posbench_$n.txt 2>&1 \
    || { echo "posbench failed ($lib)"; tail $O/posbench_$n.txt; exit 1; }
  grep "blocks     1" $O/posbench_$n.txt | sed "s/^/$n: /"
done
timeout -k 10 600 python -u tools/chain_bench.py $O/chain.json --envs 0,1,2,4,5 --repeat 3 --rounds 2 \
  --libs gym_puzzles_amd/var/libmrp_r5.so,gym_puzzles_amd/libmrp.so > $O/chain.log 2>&1 \
  || { echo "chain bench failed"; tail -20 $O/chain.log; exit 1; }
tail -2 $O/chain.log
exit 0
