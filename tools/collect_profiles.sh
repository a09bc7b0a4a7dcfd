#!/bin/bash
# Local half of tools/profile_all.sh: gpurun merges only gpurun_out/ back, so the committed
# profiles/ artefacts are rebuilt here from the merged raw rocprofv3 output.
#   tools/collect_profiles.sh <round-tag>
set -euo pipefail
R=$1
declare -A ENVS=([v0]="0 4096" [heavy_v0]="1 4096" [v2]="2 1024" [heavy_v2_3block]="4 1024" [v3]="5 4096")
for k in "${!ENVS[@]}"; do
  set -- ${ENVS[$k]}
  D=gpurun_out/prof_${R}_$k
  [ -d $D ] || continue
  python3 tools/traffic.py $D/fetch $D/write $1 $2 profiles/pmc_traffic.json
  cp "$(find $D/kt -name '*kernel_stats.csv' -print -quit)" profiles/${R}_${k}_kernel_stats.csv
  grep -h '"metric"' $D/kt.log > profiles/${R}_${k}_bench_under_rocprof.json
  python3 tools/kt_window.py "$(find $D/kt -name '*kernel_trace.csv' -print -quit)" ${WARMUP:-10} ${STEPS:-100} \
      profiles/${R}_${k}_bench_under_rocprof.json > profiles/${R}_${k}_kernel_window.json
done
grep -h '"metric"' gpurun_out/bench_default.log > profiles/${R}_bench_default.json
grep -h '"metric"' gpurun_out/bench_driver.log > profiles/${R}_bench_driver_window.json
