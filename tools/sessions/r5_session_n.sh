#!/bin/bash
# Round 5: v0 with the branch-free selection (selects form) on the lanes path only
# (var/bfl.so: -DMRP_VEL_BFREE=2 -DMRP_VEL_BFREE_LANES=1; the register paths keep the case loop)
# against the final library: slowest lane-steps alone, velbench, bench windows (interleaved).
set -uo pipefail
O=gpurun_out/r5sn
mkdir -p $O
( for i in $(seq 1 75); do date >> $O/heartbeat; sleep 15; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/chain_bench.py $O/chain.json --envs 0 --repeat 5 --rounds 2 \
    --libs gym_puzzles_amd/libmrp.so,gym_puzzles_amd/var/bfl.so > $O/chain.txt 2>&1 || { echo "chain failed"; tail $O/chain.txt; exit 1; }
tail -2 $O/chain.txt
for lib in gym_puzzles_amd/libmrp.so gym_puzzles_amd/var/bfl.so; do
  MRP_LIB=$lib timeout -k 10 120 python -u tools/velbench.py > "$O/velbench_$(basename $lib .so).txt" 2>&1 || { echo "velbench failed"; exit 1; }
  grep "blocks     1" "$O/velbench_$(basename $lib .so).txt" | sed "s/^/$(basename $lib .so): /"
done
bash tools/windows_ab.sh r5sn "gym_puzzles_amd/libmrp.so gym_puzzles_amd/var/bfl.so" || exit 1
exit 0
