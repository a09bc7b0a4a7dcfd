#!/bin/bash
# Instruction-cache counters of k_step (one PMC pass per counter pair, kernel trace only).
#   tools/pmc_icache.sh <tag> [bench args...]
set -euo pipefail
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/icache_$TAG
mkdir -p $OUT
ARGS="--steps 20 --warmup 3 --no-cpu-baseline $*"
i=0
for SET in "SQC_ICACHE_HITS SQC_ICACHE_MISSES" "SQC_ICACHE_REQ SQ_WAVES" "SQ_IFETCH SQ_WAVE_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $SET --output-format csv -d $OUT/p$i -o p$i -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1
done
python3 tools/pmc_summary.py $OUT k_step > $OUT/summary.txt
cat $OUT/summary.txt
