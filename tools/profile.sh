#!/bin/bash
# rocprofv3 passes for one bench configuration (run on the GPU box from the repo root):
#   [LANES=4096] [STEPS=100] [WARMUP=10] tools/profile.sh <tag> <env_id> [extra bench args...]
# 1) kernel trace + stats (and the mean k_step duration over exactly bench.py's timed window,
#    tools/kt_window.py), 2) PMC FETCH_SIZE, 3) PMC WRITE_SIZE -> profiles/pmc_traffic.json.
# Separate passes: counters never share a run with tracing domains other than the kernel trace.
# bench.py's diagnostics (later window, episode, multi-step, single env) are off, so the only
# k_step launches are the WARMUP untimed ones and the STEPS timed ones.
set -euo pipefail
TAG=$1; ENV=$2; shift 2
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT profiles
LANES=${LANES:-4096}
STEPS=${STEPS:-100}
WARMUP=${WARMUP:-10}
ARGS="--steps $STEPS --warmup $WARMUP --no-cpu-baseline --later-window 0 --episode 0 --multi-step 0 --single-env 0 --env $ENV --lanes $LANES $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 bench.py $ARGS > $OUT/kt.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- python3 bench.py $ARGS > $OUT/write.log 2>&1
if [ -n "${VALU_PMC:-}" ]; then   # VALU / SALU instruction counts and busy cycles (one pass, SQ block only)
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVES --output-format csv -d $OUT/valu -o valu \
      -- python3 bench.py $ARGS > $OUT/valu.log 2>&1
fi
python3 tools/traffic.py $OUT/fetch $OUT/write $ENV $LANES profiles/pmc_traffic.json
cp "$(find $OUT/kt -name '*kernel_stats.csv' -print -quit)" profiles/${TAG}_kernel_stats.csv
grep -h "\"metric\"" $OUT/kt.log > profiles/${TAG}_bench_under_rocprof.json
python3 tools/kt_window.py "$(find $OUT/kt -name '*kernel_trace.csv' -print -quit)" $WARMUP $STEPS \
    profiles/${TAG}_bench_under_rocprof.json > profiles/${TAG}_kernel_window.json
cat profiles/${TAG}_kernel_window.json
echo done
