#!/bin/bash
# PMC HBM traffic of k_step for several library builds, driver window (run on the GPU box):
#   tools/traffic_ab.sh lib.so [lib.so ...]   -> gpurun_out/traffic_<lib>.json
# FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes (tools/profile.sh's method).
set -euo pipefail
export TMPDIR=/tmp
ENV=${ENV:-0}; LANES=${LANES:-4096}; STEPS=${STEPS:-20}; WARMUP=${WARMUP:-5}
ARGS="--steps $STEPS --warmup $WARMUP --no-cpu-baseline --later-window 0 --episode 0 --multi-step 0 --single-env 0 --env $ENV --lanes $LANES ${EXTRA:-}"
for lib in "$@"; do
  n=$(basename $lib .so)
  OUT=gpurun_out/traffic_$n
  mkdir -p $OUT
  MRP_LIB=$lib timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
  MRP_LIB=$lib timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- python3 bench.py $ARGS > $OUT/write.log 2>&1
  rm -f gpurun_out/traffic_$n.json
  python3 tools/traffic.py $OUT/fetch $OUT/write $ENV $LANES gpurun_out/traffic_$n.json
  echo "$lib: $(cat gpurun_out/traffic_$n.json | tr -d '\n' | cut -c1-400)"
done
