#!/bin/bash
# Round-6 final evidence, part G (GPU box): the other configs' steady state against round 5 -- driver
# window, steps 501-700 and one whole episode of Heavy-v0, v2, the 3-block config and v3, the round-5
# library and the final one interleaved.
set -uo pipefail
O=gpurun_out/r6fg
mkdir -p $O
( for i in $(seq 1 100); do date >> $O/heartbeat; sleep 15; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
for e in 1 2 4 5; do
  L=4096; [ $e = 2 ] && L=1024; [ $e = 4 ] && L=1024
  for lib in gym_puzzles_amd/var/libmrp_r5.so gym_puzzles_amd/libmrp.so; do
    n=$(basename $lib .so)
    MRP_LIB=$lib timeout -k 10 300 python bench.py --env $e --lanes $L --steps 20 --warmup 5 --no-cpu-baseline --single-env 0 \
        --later-window 200 --episode 1 --multi-step 0 > $O/env${e}_$n.log 2>&1 || { echo "bench failed"; tail -20 $O/env${e}_$n.log; exit 1; }
    echo "env $e $n $(tail -1 $O/env${e}_$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); g=d["diagnostics"]; print(round(d["value"]/1e6,3), "M driver window,", round(g["later_window"]["env_steps_per_s"]/1e6,3), "M later,", round(g["whole_episode"]["env_steps_per_s"]/1e6,3), "M whole episode")')"
  done
done
exit 0
