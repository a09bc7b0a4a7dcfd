#!/bin/bash
# Round-6 session 9 (GPU box): two block-solver selection A/Bs against the final library -- the branch-free
# selection on the lanes path only for Heavy-v0 and v3 (libmrp_bflm.so, tools/variants/bfl_more.py) and on
# the register paths only for v3, whose TOI sub-step solve runs there (libmrp_bfr5.so,
# tools/variants/bfree_regs_v3.py): test_gpu.py with each, the slowest lane-steps alone (hashes must
# agree), driver-window lines of envs 1 and 5 interleaved.
set -uo pipefail
O=gpurun_out/r6s9
mkdir -p $O
( for i in $(seq 1 100); do date >> $O/heartbeat; sleep 15; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
for v in bflm bfr5; do
  MRP_LIB=gym_puzzles_amd/libmrp_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_$v.log 2>&1 \
    || { echo "gpu tests failed ($v)"; tail -40 $O/gpu_tests_$v.log; exit 1; }
  tail -1 $O/gpu_tests_$v.log
done
timeout -k 10 600 python -u tools/chain_bench.py $O/chain.json --envs 1,5 --repeat 3 --rounds 2 \
  --libs gym_puzzles_amd/libmrp.so,gym_puzzles_amd/libmrp_bflm.so,gym_puzzles_amd/libmrp_bfr5.so > $O/chain.log 2>&1 \
  || { echo "chain bench failed"; tail -20 $O/chain.log; exit 1; }
tail -3 $O/chain.log
for r in 0 1 2; do
  for lib in libmrp libmrp_bflm libmrp_bfr5; do
    for e in 1 5; do
      [ $lib = libmrp_bfr5 ] && [ $e = 1 ] && continue
      MRP_LIB=gym_puzzles_amd/$lib.so timeout -k 10 200 python bench.py --env $e --lanes 4096 --steps 20 --warmup 5 --no-cpu-baseline --single-env 0 \
          --later-window 0 --episode 0 --multi-step 0 > $O/cfg_${lib}_env${e}_$r.log 2>&1 || { echo "bench failed"; tail -20 $O/cfg_${lib}_env${e}_$r.log; exit 1; }
      echo "$r $lib env $e $(tail -1 $O/cfg_${lib}_env${e}_$r.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
    done
  done
done
exit 0
