#!/bin/bash
# Round-5 GPU session: [GPU suite] + chain bench (the launches' slowest lane-steps replayed alone)
# + velbench + driver-window bench, for the default library and optional variant libraries.
#   tools/sessions/r5_session.sh OUTDIR "TESTS(0/1)" "LIB1.so LIB2.so ..." [ENVS] [BENCH(0/1)]
# Every GPU step has its own time limit; the chain stops at the first failure.
set -uo pipefail
OUT=gpurun_out/$1; TESTS=$2; LIBS=$3; ENVS=${4:-0,1,2,4,5}; BENCH=${5:-1}
mkdir -p "$OUT"
( for i in $(seq 1 60); do date >> "$OUT/heartbeat"; sleep 15; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
if [ "$TESTS" = 1 ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 \
    || { echo "gpu tests failed"; tail -30 "$OUT/gpu_tests.log"; exit 1; }
  tail -1 "$OUT/gpu_tests.log"
fi
L=gym_puzzles_amd/libmrp.so
for v in $LIBS; do L="$L,$v"; done
timeout -k 10 900 python -u tools/chain_bench.py "$OUT/chain.json" --envs "$ENVS" --repeat 5 --rounds 2 --libs "$L" > "$OUT/chain.txt" 2>&1 \
  || { echo "chain bench failed"; tail -30 "$OUT/chain.txt"; exit 1; }
tail -8 "$OUT/chain.txt"
for lib in gym_puzzles_amd/libmrp.so $LIBS; do
  MRP_LIB=$lib timeout -k 10 120 python -u tools/velbench.py > "$OUT/velbench_$(basename $lib .so).txt" 2>&1 \
    || { echo "velbench failed ($lib)"; tail "$OUT/velbench_$(basename $lib .so).txt"; exit 1; }
  grep "blocks     1" "$OUT/velbench_$(basename $lib .so).txt" | sed "s/^/$(basename $lib .so): /"
done
for lib in gym_puzzles_amd/libmrp.so $LIBS; do
  MRP_LIB=$lib timeout -k 10 120 python -u tools/posbench.py > "$OUT/posbench_$(basename $lib .so).txt" 2>&1 \
    || { echo "posbench failed ($lib)"; tail "$OUT/posbench_$(basename $lib .so).txt"; exit 1; }
  grep "blocks     1" "$OUT/posbench_$(basename $lib .so).txt" | sed "s/^/$(basename $lib .so): /"
done
if [ "$BENCH" = 1 ]; then
  for lib in gym_puzzles_amd/libmrp.so $LIBS; do
    MRP_LIB=$lib timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --single-env 0 --later-window 0 --episode 0 --multi-step 0 > "$OUT/bench_drv_$(basename $lib .so).log" 2>&1 \
      || { echo "bench failed ($lib)"; tail -20 "$OUT/bench_drv_$(basename $lib .so).log"; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'driver window', round(d['value']/1e6,3), 'M env-steps/s kernel_ms', round(d['roofline']['kernel_ms'],4))" "$OUT/bench_drv_$(basename $lib .so).log" "$(basename $lib .so)"
  done
fi
