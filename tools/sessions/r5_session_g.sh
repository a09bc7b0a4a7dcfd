#!/bin/bash
# Round 5: (a) v0 two-body register path gated on the lane's cost priority (var/xg.so:
# -DMRP_XW_LATE=32 -DMRP_XW_GATE=3, run with mrp_set_schedule(2)) against the default library with
# and without cost priority: bench windows interleaved, then PMC traffic; (b) v3 with
# MRP_FRESH_REGS (var/fr5.so): slowest lane-steps alone, driver window, PMC traffic.
set -uo pipefail
O=gpurun_out/r5sg
mkdir -p $O
( for i in $(seq 1 75); do date >> $O/heartbeat; sleep 15; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
bash tools/windows_ab_args.sh r5sg "base=gym_puzzles_amd/libmrp.so" "base_s2=gym_puzzles_amd/libmrp.so:--schedule,2" \
    "xg_s2=gym_puzzles_amd/var/xg.so:--schedule,2" || exit 1
EXTRA="--schedule 2" bash tools/traffic_ab.sh gym_puzzles_amd/var/xg.so > $O/traffic_xg.txt 2>&1 || { echo "traffic xg failed"; exit 1; }
tail -1 $O/traffic_xg.txt | cut -c1-200
timeout -k 10 500 python -u tools/chain_bench.py $O/chain.json --envs 5 --repeat 5 --rounds 2 \
    --libs gym_puzzles_amd/libmrp.so,gym_puzzles_amd/var/fr5.so > $O/chain.txt 2>&1 || { echo "chain failed"; tail $O/chain.txt; exit 1; }
tail -2 $O/chain.txt
for r in 0 1; do for lib in gym_puzzles_amd/libmrp.so gym_puzzles_amd/var/fr5.so; do
  MRP_LIB=$lib timeout -k 10 200 python bench.py --env 5 --lanes 4096 --steps 20 --warmup 5 --no-cpu-baseline --single-env 0 --later-window 0 --episode 0 --multi-step 0 \
      > $O/drv5_$(basename $lib .so)_$r.log 2>&1 || { echo "bench failed"; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']/1e6,3))" $O/drv5_$(basename $lib .so)_$r.log "round $r v3 $(basename $lib .so)"
done; done
ENV=5 bash tools/traffic_ab.sh gym_puzzles_amd/libmrp.so gym_puzzles_amd/var/fr5.so > $O/traffic5.txt 2>&1 || { echo "traffic 5 failed"; exit 1; }
grep "^gym" $O/traffic5.txt | cut -c1-200
exit 0
