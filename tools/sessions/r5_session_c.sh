#!/bin/bash
# Round 5: v0 with the two-ballot case test and the cross-product tangent speed (var/v5.so) against
# the default library (slowest lane-steps alone, then the three bench windows, interleaved), and the
# rocprofv3 sets of v2 and the 3-block config on this round's library (their units changed).
set -uo pipefail
O=gpurun_out/r5sc
mkdir -p $O
( for i in $(seq 1 75); do date >> $O/heartbeat; sleep 15; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/chain_bench.py $O/chain.json --envs 0 --repeat 5 --rounds 2 \
    --libs gym_puzzles_amd/libmrp.so,gym_puzzles_amd/var/v5.so > $O/chain.txt 2>&1 || { echo "chain failed"; tail $O/chain.txt; exit 1; }
tail -3 $O/chain.txt
bash tools/windows_ab.sh r5sc "gym_puzzles_amd/libmrp.so gym_puzzles_amd/var/v5.so" || exit 1
STEPS=20 WARMUP=5 LANES=1024 timeout -k 10 400 bash tools/profile.sh r5_v2 2 > /dev/null || { echo "profile 2 failed"; exit 1; }
STEPS=20 WARMUP=5 LANES=1024 timeout -k 10 400 bash tools/profile.sh r5_heavy_v2_3block 4 > /dev/null || { echo "profile 4 failed"; exit 1; }
echo profiles done
exit 0
