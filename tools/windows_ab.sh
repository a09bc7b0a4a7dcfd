#!/bin/bash
# v0 bench windows per library, interleaved over two rounds (GPU box):
#   tools/windows_ab.sh OUTDIR "LIB1.so LIB2.so ..."
# driver window (steps 6-25), bench default (steps 21-220), the later window (steps 501-700) and one
# whole episode; each run under
# its own time limit, the first failure ends the script.
set -uo pipefail
OUT=gpurun_out/$1; LIBS=$2
mkdir -p "$OUT"
for r in 0 1; do
  for lib in $LIBS; do
    n=$(basename $lib .so)
    MRP_LIB=$lib timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --single-env 0 --later-window 0 --episode 0 --multi-step 0 > "$OUT/drv_${n}_$r.log" 2>&1 \
      || { echo "bench failed ($lib)"; tail -20 "$OUT/drv_${n}_$r.log"; exit 1; }
    MRP_LIB=$lib timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --single-env 0 --later-window 200 --episode 1 --multi-step 0 > "$OUT/def_${n}_$r.log" 2>&1 \
      || { echo "bench failed ($lib)"; tail -20 "$OUT/def_${n}_$r.log"; exit 1; }
    python - "$OUT/drv_${n}_$r.log" "$OUT/def_${n}_$r.log" "$n" "$r" <<'PY'
import json, sys
a = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
b = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ep = b.get("diagnostics", b).get("whole_episode") or {}
epv = ep.get("env_steps_per_s")
lw = (b.get("diagnostics", b).get("later_window") or {}).get("env_steps_per_s")
print(f"round {sys.argv[4]} {sys.argv[3]:10s} driver window {a['value'] / 1e6:7.3f} M  steps 21-220 {b['value'] / 1e6:7.3f} M  "
      f"later window {lw / 1e6 if lw else float('nan'):7.3f} M  whole episode {epv / 1e6 if epv else float('nan'):7.3f} M", flush=True)
PY
  done
done
