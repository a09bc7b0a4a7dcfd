#!/bin/bash
# rocprofv3 passes for one bench configuration (run on the GPU box from the repo root).
#   tools/profile.sh <tag> [bench args...]
# 1) kernel trace + stats, 2) PMC FETCH_SIZE, 3) PMC WRITE_SIZE, 4) PMC instruction mix.
# Separate passes: counters never share a run with tracing domains other than the kernel trace.
set -euo pipefail
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
ARGS="--steps 50 --warmup 5 --no-cpu-baseline $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 bench.py $ARGS > $OUT/kt.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- python3 bench.py $ARGS > $OUT/write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/inst -o inst -- python3 bench.py $ARGS > $OUT/inst.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_FLAT SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d $OUT/inst2 -o inst2 -- python3 bench.py $ARGS > $OUT/inst2.log 2>&1
echo done
