#!/bin/bash
# A/B of mrp_set_schedule modes on the GPU box: tools/ab_sched.sh mode... (bench 20/5 and 200/20, twice each, interleaved)
set -uo pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_sched.txt; : > $out
for rep in 1 2; do
  for m in "$@"; do
    for cfg in "20 5" "200 20"; do
      read -r K W <<< "$cfg"
      r=$(timeout -k 5 120 python bench.py --steps $K --warmup $W --no-cpu-baseline --later-window 0 --schedule $m 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.3fM' % (d['value']/1e6), 'kernel %.3f ms' % d['roofline']['kernel_ms'])") || { echo "bench failed for mode $m"; exit 1; }
      echo "schedule=$m steps=$K warmup=$W: $r" | tee -a $out
    done
  done
done
