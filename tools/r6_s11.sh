#!/bin/bash
# Round-6 session 11 (GPU box): v0 and v3 at 4 waves per SIMD (libmrp_w4.so, tools/variants/w4_v0_v3.py)
# against the final library: test_gpu.py with the variant, the slowest lane-steps alone (hashes must
# agree), v0's four windows interleaved, v3's driver window, later window and whole episode interleaved.
set -uo pipefail
O=gpurun_out/r6s11
mkdir -p $O
( for i in $(seq 1 100); do date >> $O/heartbeat; sleep 15; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
MRP_LIB=gym_puzzles_amd/libmrp_w4.so timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -x -q -k "not costliest_first_schedule" --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  || { echo "gpu tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 600 python -u tools/chain_bench.py $O/chain.json --envs 0,5 --repeat 3 --rounds 2 \
  --libs gym_puzzles_amd/libmrp.so,gym_puzzles_amd/libmrp_w4.so > $O/chain.log 2>&1 \
  || { echo "chain bench failed"; tail -20 $O/chain.log; exit 1; }
tail -2 $O/chain.log
timeout -k 10 700 bash tools/windows_ab.sh r6s11/win "gym_puzzles_amd/libmrp.so gym_puzzles_amd/libmrp_w4.so" || { echo "windows failed"; exit 1; }
for r in 0 1; do
  for lib in libmrp libmrp_w4; do
    MRP_LIB=gym_puzzles_amd/$lib.so timeout -k 10 200 python bench.py --env 5 --lanes 4096 --steps 20 --warmup 5 --no-cpu-baseline --single-env 0 \
        --later-window 200 --episode 1 --multi-step 0 > $O/cfg_${lib}_env5_$r.log 2>&1 || { echo "bench failed"; tail -20 $O/cfg_${lib}_env5_$r.log; exit 1; }
    echo "$r $lib env 5 $(tail -1 $O/cfg_${lib}_env5_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); g=d["diagnostics"]; print(round(d["value"]/1e6,3), "M driver window,", round(g["later_window"]["env_steps_per_s"]/1e6,3), "M later,", round(g["whole_episode"]["env_steps_per_s"]/1e6,3), "M whole episode")')"
  done
done
exit 0
