#!/bin/bash
# Round-4 session 10: the stamps build without in-kernel atomics (k_stamp_fold after the launch):
# the lane timeline of v0 and v3 at 4096 lanes with and without costliest-first dispatch, and the
# per-phase split of every config's driver window (regenerates profiles/r4_phase_env*).
set -uo pipefail
O=gpurun_out/r4s10
mkdir -p $O
( for i in $(seq 1 80); do date >> gpurun_out/heartbeat; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
export MRP_LIB=gym_puzzles_amd/libmrp_stamps.so
for env in 0 5; do
  for s in 0 1; do
    MRP_SCHEDULE=$s timeout -k 10 200 python tools/lane_phases.py $env 4096 5 20 $O/lanes_env${env}_s$s.json > $O/lanes_env${env}_s$s.txt 2>&1 \
      || { echo "lane_phases env $env failed"; tail $O/lanes_env${env}_s$s.txt; exit 1; }
    echo "== env $env schedule $s"; cat $O/lanes_env${env}_s$s.txt
  done
done
for cfg in 0:4096 1:4096 2:1024 4:1024 5:4096; do
  env=${cfg%%:*}; lanes=${cfg##*:}
  timeout -k 10 200 python tools/phase_profile.py $env $lanes 5 20 $O/r4_phase_env$env.json > $O/r4_phase_env$env.txt 2>&1 \
    || { echo "phase_profile env $env failed"; tail $O/r4_phase_env$env.txt; exit 1; }
  cat $O/r4_phase_env$env.txt
done
exit 0
