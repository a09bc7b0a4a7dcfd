#!/bin/bash
# Round 5: the branch-free case selection with the "any case holds" test as per-lane selects too
# (var/bf2.so: -DMRP_VEL_BFREE=2 for v0, v2 and the 3-block config) against the final library:
# slowest lane-steps alone, velbench, v0's bench windows, v2 / 3-block driver windows (interleaved).
set -uo pipefail
O=gpurun_out/r5sk
mkdir -p $O
( for i in $(seq 1 75); do date >> $O/heartbeat; sleep 15; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/chain_bench.py $O/chain.json --envs 0,2,4 --repeat 5 --rounds 2 \
    --libs gym_puzzles_amd/libmrp.so,gym_puzzles_amd/var/bf2.so > $O/chain.txt 2>&1 || { echo "chain failed"; tail $O/chain.txt; exit 1; }
tail -2 $O/chain.txt
for lib in gym_puzzles_amd/libmrp.so gym_puzzles_amd/var/bf2.so; do
  MRP_LIB=$lib timeout -k 10 120 python -u tools/velbench.py > "$O/velbench_$(basename $lib .so).txt" 2>&1 || { echo "velbench failed"; exit 1; }
  grep "blocks     1" "$O/velbench_$(basename $lib .so).txt" | sed "s/^/$(basename $lib .so): /"
done
bash tools/windows_ab.sh r5sk "gym_puzzles_amd/libmrp.so gym_puzzles_amd/var/bf2.so" || exit 1
for r in 0 1; do for e in 2 4; do for lib in gym_puzzles_amd/libmrp.so gym_puzzles_amd/var/bf2.so; do
  MRP_LIB=$lib timeout -k 10 200 python bench.py --env $e --lanes 1024 --steps 20 --warmup 5 --no-cpu-baseline --single-env 0 --later-window 0 --episode 0 --multi-step 0 \
      > $O/drv${e}_$(basename $lib .so)_$r.log 2>&1 || { echo "bench failed"; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']/1e6,3))" $O/drv${e}_$(basename $lib .so)_$r.log "round $r env $e $(basename $lib .so)"
done; done; done
exit 0
