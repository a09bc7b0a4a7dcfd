#!/bin/bash
# Round-6 session 2b (GPU box): v0 bench windows (driver window, steps 21-220, 501-700, whole episode) of
# the round-5 library, its PICK2_VT / BFREE_LANES A/B builds and the new library, interleaved.
set -uo pipefail
O=gpurun_out/r6s2
mkdir -p $O
( for i in $(seq 1 80); do date >> $O/heartbeat_b; sleep 15; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
timeout -k 10 1100 bash tools/windows_ab.sh r6s2/win "gym_puzzles_amd/var/libmrp_r5.so gym_puzzles_amd/libmrp_ab_v0_nopick.so gym_puzzles_amd/libmrp_ab_v0_nobfl.so gym_puzzles_amd/libmrp_ab_v0_neither.so gym_puzzles_amd/libmrp.so gym_puzzles_amd/libmrp_r6b.so" \
  || { echo "windows failed"; exit 1; }
exit 0
