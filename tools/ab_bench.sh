#!/bin/bash
# A/B of library builds (and schedule modes) on the GPU box, bench 20/5 and 200/20, twice each, interleaved:
#   [ENV=0] [LANES=4096] tools/ab_bench.sh libA.so[:mode] libB.so[:mode] ...
set -uo pipefail
ENV=${ENV:-0}; LANES=${LANES:-4096}
mkdir -p gpurun_out
out=gpurun_out/ab.txt; [ "$ENV" != 0 ] && out=gpurun_out/ab_env$ENV.txt; : > $out
for rep in 1 2; do
  for spec in "$@"; do
    lib=${spec%%:*}; mode=0
    [[ "$spec" == *:* ]] && mode=${spec##*:}
    for cfg in "20 5" "200 20"; do
      read -r K W <<< "$cfg"
      r=$(MRP_LIB=$lib timeout -k 5 120 python bench.py --env $ENV --lanes $LANES --steps $K --warmup $W --no-cpu-baseline --later-window 0 --episode 0 --multi-step 0 --single-env 0 --schedule $mode 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.3fM' % (d['value']/1e6), 'kernel %.3f ms' % d['roofline']['kernel_ms'])") || { echo "bench failed for $spec"; exit 1; }
      echo "$spec env=$ENV lanes=$LANES steps=$K warmup=$W: $r" | tee -a $out
    done
  done
done
