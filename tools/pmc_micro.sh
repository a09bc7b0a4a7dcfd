#!/bin/bash
# SQ instruction counters of the micro-benchmarks and of the chain replays (one library):
#   tools/pmc_micro.sh OUTDIR [LIB]
# One rocprofv3 --pmc pass per program, under its own time limit; stops at the first failure.
set -uo pipefail
OUT=gpurun_out/$1; LIB=${2:-gym_puzzles_amd/libmrp.so}
mkdir -p "$OUT"
export MRP_LIB=$LIB
SET="SQ_INSTS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_WAVE_CYCLES"
timeout -s KILL 120 rocprofv3 --pmc $SET --output-format csv -d "$OUT/pv" -o pv -- python3 tools/velbench.py > "$OUT/pv.log" 2>&1 || { echo "pmc velbench failed"; tail "$OUT/pv.log"; exit 1; }
python3 tools/pmc_micro.py "$OUT/pv/pv_counter_collection.csv" velbench
timeout -s KILL 120 rocprofv3 --pmc $SET --output-format csv -d "$OUT/pp" -o pp -- python3 tools/posbench.py > "$OUT/pp.log" 2>&1 || { echo "pmc posbench failed"; tail "$OUT/pp.log"; exit 1; }
python3 tools/pmc_micro.py "$OUT/pp/pp_counter_collection.csv" posbench
grep "blocks     1" "$OUT/pp.log"
timeout -s KILL 200 rocprofv3 --pmc $SET --output-format csv -d "$OUT/pc" -o pc -- python3 tools/chain_bench.py "$OUT/pc.json" --envs 0,2,4 --repeat 1 --child > "$OUT/pc.log" 2>&1 || { echo "pmc chain failed"; tail "$OUT/pc.log"; exit 1; }
echo "chain replays under counters done"
