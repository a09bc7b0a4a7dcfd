#!/bin/bash
# Cost of the per-step HIP timing events: bench with events on every step vs only the first.
for rep in 1 2; do for te in 1 1000000; do for cfg in "20 5" "200 20"; do read -r K W <<< "$cfg"; r=$(timeout -k 5 120 python bench.py --steps $K --warmup $W --no-cpu-baseline --later-window 0 --episode 0 --time-every $te 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.3fM' % (d['value']/1e6), 'ms/step %.4f' % d['ms_per_step'], 'kernel %.4f' % d['roofline']['kernel_ms'])"); echo "te=$te K=$K: $r"; done; done; done
