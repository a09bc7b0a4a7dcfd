#!/bin/bash
# Slowest-lane replays (stamps build) with island topologies:  tools/topo_replay.sh <env> <lanes> <warm>...
set -uo pipefail
mkdir -p gpurun_out
ENV=$1; LANES=$2; shift 2
for w in "$@"; do
  MRP_LIB=gym_puzzles_amd/libmrp_stamps.so timeout -k 10 100 python tools/lane_replay.py $ENV $LANES $w 6 > gpurun_out/topo_${ENV}_$w.txt 2>&1 || exit 1
  echo "== env $ENV lanes $LANES warm $w"; cat gpurun_out/topo_${ENV}_$w.txt
done
