#!/bin/bash
# Round-6 session 1b (GPU box): posbench of the no-memo diagnostic, v0 / Heavy-v0 phase tables on the
# round-5 code (stamps build), the RCCL one-rank test, single-env timing per spawn seed.
set -uo pipefail
O=gpurun_out/r6s1b
mkdir -p $O
( for i in $(seq 1 80); do date >> $O/heartbeat; sleep 15; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
for lib in libmrp_d_nomemo libmrp_ab_v0_nopick; do
  [ -f gym_puzzles_amd/$lib.so ] || continue
  MRP_LIB=gym_puzzles_amd/$lib.so timeout -k 10 120 python -u tools/posbench.py > $O/posbench_$lib.txt 2>&1 \
    || { echo "posbench failed ($lib)"; tail $O/posbench_$lib.txt; exit 1; }
  grep "blocks     1" $O/posbench_$lib.txt | sed "s/^/$lib: /"
done
for e in 0 1; do
  MRP_LIB=gym_puzzles_amd/var/stamps_r6.so timeout -k 10 200 python tools/phase_profile.py $e 4096 5 20 $O/phase_env$e.json > $O/phase_env$e.txt 2>&1 \
    || { echo "phase $e failed"; tail $O/phase_env$e.txt; exit 1; }
  head -20 $O/phase_env$e.txt
done
timeout -k 10 300 python -u -m pytest tests/test_dist_gpu.py -x -v --timeout 280 --timeout-method thread > $O/dist_gpu.log 2>&1 \
  || { echo "dist gpu tests failed"; tail -40 $O/dist_gpu.log; exit 1; }
tail -3 $O/dist_gpu.log
timeout -k 10 200 python - > $O/single_env.json 2>$O/single_env.err <<'PY'
import json, sys
sys.path.insert(0, ".")
import bench
for rep in range(2):
    r = bench.single_env_rate(0, 300, seeds=(0, 1, 2, 3, 4, 5, 6, 7))
    print(json.dumps(r), flush=True)
PY
[ $? -eq 0 ] || { echo "single env failed"; tail $O/single_env.err; exit 1; }
python - $O/single_env.json <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    r = json.loads(ln)
    print("mean %.1f us/step;" % r["us_per_step"], " ".join("s%d %.1f us (%.2f touching, %.1f pos it)" % (p["seed"], p["us_per_step"], p["touching_contacts_per_step"], p["position_iterations_per_step"]) for p in r["per_seed"]))
PY
exit 0
