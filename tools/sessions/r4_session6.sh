#!/bin/bash
# Round-4 session 6: Heavy-v0 (env 1) with and without its out-of-line max-ilp lanes loops on the
# one-call-site k_step (register count decides its occupancy), and memory-latency / TLB counters of
# the v0 driver window at 4096 lanes (late-dispatched lanes) against 2048 (none).
set -uo pipefail
O=gpurun_out/r4s6
mkdir -p $O
( for i in $(seq 1 80); do date >> gpurun_out/heartbeat; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --later-window 200 --later-start 21 --episode 1 --multi-step 0 --single-env 0"
for round in 1 2; do
  for lib in libmrp libmrp_e1plain libmrp_e1w2 libmrp_e1w2p libmrp_old; do
    MRP_LIB=gym_puzzles_amd/$lib.so timeout -k 10 200 python bench.py --env 1 $ARGS > $O/ab_${lib}_env1_r$round.log 2>&1 \
      || { echo "bench $lib failed"; tail $O/ab_${lib}_env1_r$round.log; exit 1; }
    python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; g=d['diagnostics']; print('env 1', sys.argv[2], round(d['value']/1e6,3), 'M/s window; later', round(g['later_window']['env_steps_per_s']/1e6,3), 'episode', round(g['whole_episode']['env_steps_per_s']/1e6,3), 'kernel_ms', round(d['roofline']['kernel_ms'],4))" $O/ab_${lib}_env1_r$round.log $lib
  done
done
B="--env 0 --steps 20 --warmup 5 --no-cpu-baseline --later-window 0 --episode 0 --multi-step 0 --single-env 0"
i=0
for L in 4096 2048; do
  for SET in "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum" \
             "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TCP_PENDING_STALL_CYCLES_sum TCP_UTCL1_SERIALIZATION_STALL_sum" \
             "TCC_EA0_WRREQ_STALL_sum TCC_TAG_STALL_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $SET --output-format csv -d $O/mem_L${L}_p$i -o p -- python3 bench.py $B --lanes $L > $O/mem_L${L}_p$i.log 2>&1 \
      || { echo "pmc pass $i failed"; tail $O/mem_L${L}_p$i.log; exit 1; }
  done
  echo "lanes $L"; python3 tools/pmc_summary.py "$O" k_step > /dev/null
  for d in $O/mem_L${L}_p*; do python3 tools/pmc_summary.py $d k_step; done
done
exit 0
