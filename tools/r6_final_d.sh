#!/bin/bash
# Round-6 final evidence, part D (GPU box): the slowest lane-steps alone of the round-5 library, the final
# one and the final one with the rotation memo in v0 / Heavy-v0 (libmrp_noonerot.so, MRP_ONE_ROT=0 on
# their units), then those two envs' driver-window lines of the final library with and without ONE_ROT,
# interleaved, with v0's thread id made opaque per island / TOI pass (libmrp_ftid.so, tools/variants/fresh_tid.py;
# also its PMC traffic) and Heavy-v0 held to 2 waves per SIMD (libmrp_heavyw2.so, MRP_STEP_WAVES_PER_EU=2 on its unit).
set -uo pipefail
O=gpurun_out/r6fd
mkdir -p $O
( for i in $(seq 1 100); do date >> $O/heartbeat; sleep 15; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
timeout -k 10 700 python -u tools/chain_bench.py $O/chain.json --envs 0,1,2,4,5 --repeat 3 --rounds 2 \
  --libs gym_puzzles_amd/var/libmrp_r5.so,gym_puzzles_amd/libmrp.so,gym_puzzles_amd/libmrp_noonerot.so,gym_puzzles_amd/libmrp_ftid.so > $O/chain.log 2>&1 \
  || { echo "chain bench failed"; tail -20 $O/chain.log; exit 1; }
tail -4 $O/chain.log
for r in 0 1; do
  for lib in libmrp libmrp_noonerot libmrp_heavyw2 libmrp_ftid; do
    for e in 0 1; do
      [ $lib = libmrp_heavyw2 ] && [ $e = 0 ] && continue
      [ $lib = libmrp_ftid ] && [ $e = 1 ] && continue
      MRP_LIB=gym_puzzles_amd/$lib.so timeout -k 10 200 python bench.py --env $e --lanes 4096 --steps 20 --warmup 5 --no-cpu-baseline --single-env 0 \
          --later-window 0 --episode 0 --multi-step 0 > $O/ab_${lib}_env${e}_$r.log 2>&1 || { echo "bench failed"; tail -20 $O/ab_${lib}_env${e}_$r.log; exit 1; }
      echo "$r $lib env $e $(tail -1 $O/ab_${lib}_env${e}_$r.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
    done
  done
done
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --later-window 0 --episode 0 --multi-step 0 --single-env 0 --env 0 --lanes 4096"
MRP_LIB=gym_puzzles_amd/libmrp_ftid.so timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/ftid_fetch -o fetch -- python3 bench.py $ARGS > $O/ftid_fetch.log 2>&1 \
  || { echo "fetch pass failed"; tail $O/ftid_fetch.log; exit 1; }
MRP_LIB=gym_puzzles_amd/libmrp_ftid.so timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/ftid_write -o write -- python3 bench.py $ARGS > $O/ftid_write.log 2>&1 \
  || { echo "write pass failed"; tail $O/ftid_write.log; exit 1; }
python3 tools/traffic.py $O/ftid_fetch $O/ftid_write 0 4096 $O/ftid_traffic.json
exit 0
