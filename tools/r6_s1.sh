#!/bin/bash
# Round-6 session 1 (GPU box): position-pass measurements and the RCCL one-rank test.
#  - f64 / rot dependent-chain costs (tools/micro/f64lat)
#  - posbench on the default library and the diagnostic decompositions (cheap rot, no memo, fast div)
#  - SQ instruction counters of posbench (instructions per point update)
#  - phase tables of v0 / Heavy-v0 on the stamps build (position_passes baseline)
#  - the new -m gpu RCCL test (bench.py --force-collective under torch.distributed.run)
set -uo pipefail
O=gpurun_out/r6s1
mkdir -p $O
( for i in $(seq 1 80); do date >> $O/heartbeat; sleep 15; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
timeout -k 10 60 ./tools/micro/f64lat > $O/f64lat.txt 2>&1 || { echo "f64lat failed"; cat $O/f64lat.txt; exit 1; }
cat $O/f64lat.txt
for lib in libmrp libmrp_d_cheaprot libmrp_d_nomemo libmrp_d_fastdiv; do
  [ -f gym_puzzles_amd/$lib.so ] || continue
  MRP_LIB=gym_puzzles_amd/$lib.so timeout -k 10 120 python -u tools/posbench.py > $O/posbench_$lib.txt 2>&1 \
    || { echo "posbench failed ($lib)"; tail $O/posbench_$lib.txt; exit 1; }
  grep "blocks     1" $O/posbench_$lib.txt | sed "s/^/$lib: /"
done
SET="SQ_INSTS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_WAVE_CYCLES"
timeout -s KILL 120 rocprofv3 --pmc $SET --output-format csv -d $O/pp -o pp -- python3 tools/posbench.py > $O/pp.log 2>&1 \
  || { echo "pmc posbench failed"; tail $O/pp.log; exit 1; }
python3 tools/pmc_micro.py $O/pp/pp_counter_collection.csv posbench | tee $O/pp_insts.txt
for e in 0 1; do
  MRP_LIB=gym_puzzles_amd/libmrp_stamps.so timeout -k 10 200 python tools/phase_profile.py $e 4096 5 20 $O/phase_env$e.json > $O/phase_env$e.txt 2>&1 \
    || { echo "phase $e failed"; tail $O/phase_env$e.txt; exit 1; }
  head -20 $O/phase_env$e.txt
done
timeout -k 10 300 python -u -m pytest tests/test_dist_gpu.py -x -v --timeout 280 --timeout-method thread > $O/dist_gpu.log 2>&1 \
  || { echo "dist gpu tests failed"; tail -40 $O/dist_gpu.log; exit 1; }
tail -3 $O/dist_gpu.log
exit 0
