#!/bin/bash
# Round-6 session 6 (GPU box): rot() with the straight-line fast form first and glibc's large-argument
# branch behind a wave-uniform test (libmrp_rotlate.so: envs 0, 1, 2, 4, 5 from tools/variants/rot_late.py,
# the rest the default library) against the default library: the step-parity tests, the slowest
# lane-steps alone (hashes must agree), driver-window config lines interleaved.
set -uo pipefail
O=gpurun_out/r6s6
mkdir -p $O
( for i in $(seq 1 80); do date >> $O/heartbeat; sleep 15; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
MRP_LIB=gym_puzzles_amd/libmrp_rotlate.so timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  || { echo "gpu tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 700 python -u tools/chain_bench.py $O/chain.json --envs 0,1,2,4,5 --repeat 3 --rounds 2 \
  --libs gym_puzzles_amd/libmrp.so,gym_puzzles_amd/libmrp_rotlate.so > $O/chain.log 2>&1 \
  || { echo "chain bench failed"; tail -20 $O/chain.log; exit 1; }
tail -3 $O/chain.log
for r in 0 1; do
  for lib in libmrp libmrp_rotlate; do
    for e in 0 1 2 4 5; do
      L=4096; [ $e = 2 ] && L=1024; [ $e = 4 ] && L=1024
      MRP_LIB=gym_puzzles_amd/$lib.so timeout -k 10 200 python bench.py --env $e --lanes $L --steps 20 --warmup 5 --no-cpu-baseline --single-env 0 \
          --later-window 0 --episode 0 --multi-step 0 > $O/cfg_${lib}_env${e}_$r.log 2>&1 || { echo "bench failed"; tail -20 $O/cfg_${lib}_env${e}_$r.log; exit 1; }
      echo "$r $lib env $e $(tail -1 $O/cfg_${lib}_env${e}_$r.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
    done
  done
done
exit 0
