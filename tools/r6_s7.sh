#!/bin/bash
# Round-6 session 7 (GPU box): MRP_FRESH_REGS on the Heavy-v0, v2 and 3-block units (libmrp_fmore.so,
# tools/variants/fresh_more.py) against the final library: test_gpu.py with the variant, the slowest
# lane-steps alone (hashes must agree), driver-window config lines of envs 1, 2, 4 interleaved.
set -uo pipefail
O=gpurun_out/r6s7
mkdir -p $O
( for i in $(seq 1 100); do date >> $O/heartbeat; sleep 15; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
MRP_LIB=gym_puzzles_amd/libmrp_fmore.so timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  || { echo "gpu tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 600 python -u tools/chain_bench.py $O/chain.json --envs 1,2,4 --repeat 3 --rounds 2 \
  --libs gym_puzzles_amd/libmrp.so,gym_puzzles_amd/libmrp_fmore.so > $O/chain.log 2>&1 \
  || { echo "chain bench failed"; tail -20 $O/chain.log; exit 1; }
tail -2 $O/chain.log
for r in 0 1 2; do
  for lib in libmrp libmrp_fmore; do
    for e in 1 2 4; do
      L=4096; [ $e = 2 ] && L=1024; [ $e = 4 ] && L=1024
      MRP_LIB=gym_puzzles_amd/$lib.so timeout -k 10 200 python bench.py --env $e --lanes $L --steps 20 --warmup 5 --no-cpu-baseline --single-env 0 \
          --later-window 0 --episode 0 --multi-step 0 > $O/cfg_${lib}_env${e}_$r.log 2>&1 || { echo "bench failed"; tail -20 $O/cfg_${lib}_env${e}_$r.log; exit 1; }
      echo "$r $lib env $e $(tail -1 $O/cfg_${lib}_env${e}_$r.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
    done
  done
done
exit 0
