#!/bin/bash
# Round-4 session 12: the out-of-line, ILP-scheduled lanes-path loops of Heavy-v0 (env 1) and the
# 3-block config (env 4) against the same loops inlined (with and without the max-ilp scheduler):
# driver-window A/B and the PMC traffic per launch of each (FETCH_SIZE x2 + WRITE_SIZE, separate
# passes, MI355X_MICROARCH.md).  libmrp.so = default (noinline + max-ilp), libmrp_e14inl.so =
# inline + max-ilp, libmrp_e14plain.so = inline, default scheduler; libmrp_lp.so = the lanes-path
# sweeps two per loop trip (-DMRP_LANES_PAIRS=1, envs 0 1 4 5), A/B'd on v0 and v3 too.
set -uo pipefail
O=gpurun_out/r4s12
mkdir -p $O
( for i in $(seq 1 80); do date >> gpurun_out/heartbeat; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
T=tests/test_gpu.py
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests_default.log 2>&1 \
  || { echo "gpu suite failed (default library)"; tail -30 $O/tests_default.log; exit 1; }
echo "default library, GPU suite: $(tail -1 $O/tests_default.log)"
for lib in libmrp_e14inl libmrp_e14plain libmrp_lp; do
  MRP_LIB=gym_puzzles_amd/$lib.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
      "$T::test_device_autoreset_full_size[1]" "$T::test_device_autoreset_full_size[4]" "$T::test_step_parity_host_inputs[1]" \
      "$T::test_step_parity_host_inputs[4]" "$T::test_whole_episode_soak[4]" "$T::test_device_autoreset_full_size[0]" "$T::test_whole_episode_soak[0]" "$T::test_device_autoreset_full_size[5]" > $O/tests_$lib.log 2>&1 \
    || { echo "gpu tests failed ($lib)"; tail -30 $O/tests_$lib.log; exit 1; }
  echo "$lib parity: $(tail -1 $O/tests_$lib.log)"
done
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --later-window 200 --later-start 21 --episode 0 --multi-step 0 --single-env 0"
for round in 1 2; do
  for cfg in 1:4096 4:1024 0:4096 5:4096; do
    env=${cfg%%:*}; lanes=${cfg##*:}
    libs="libmrp libmrp_e14inl libmrp_e14plain libmrp_lp"; [ $env = 0 -o $env = 5 ] && libs="libmrp libmrp_lp"
    for lib in $libs; do
      MRP_LIB=gym_puzzles_amd/$lib.so timeout -k 10 200 python bench.py --env $env --lanes $lanes $ARGS > $O/ab_${lib}_env${env}_r$round.log 2>&1 \
        || { echo "bench $lib env $env failed"; tail $O/ab_${lib}_env${env}_r$round.log; exit 1; }
      python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; g=d['diagnostics']; print('env', sys.argv[3], sys.argv[2], round(d['value']/1e6,3), 'M/s window; later', round(g['later_window']['env_steps_per_s']/1e6,3), 'kernel_ms', round(d['roofline']['kernel_ms'],4))" \
        $O/ab_${lib}_env${env}_r$round.log $lib $env
    done
  done
done
B="--steps 20 --warmup 5 --no-cpu-baseline --later-window 0 --episode 0 --multi-step 0 --single-env 0"
for cfg in 1:4096 4:1024; do
  env=${cfg%%:*}; lanes=${cfg##*:}
  for lib in libmrp libmrp_e14inl libmrp_e14plain; do
    for c in FETCH_SIZE WRITE_SIZE; do
      MRP_LIB=gym_puzzles_amd/$lib.so timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_${lib}_env${env}_$c -o p \
          -- python3 bench.py $B --env $env --lanes $lanes > $O/pmc_${lib}_env${env}_$c.log 2>&1 \
        || { echo "pmc $c $lib env $env failed"; tail $O/pmc_${lib}_env${env}_$c.log; exit 1; }
    done
    python3 tools/traffic.py $O/pmc_${lib}_env${env}_FETCH_SIZE $O/pmc_${lib}_env${env}_WRITE_SIZE $env $lanes $O/traffic_$lib.json > /dev/null
    python3 -c "import json,sys; d=json.load(open(sys.argv[1]))[sys.argv[2]]; print('env', sys.argv[2], sys.argv[3], 'traffic MB/launch', round(d['hbm_bytes_per_launch']/1e6, 2), 'fetch', round(d['fetch_bytes_per_launch']/1e6, 2), 'write', round(d['write_bytes_per_launch']/1e6, 2))" \
      $O/traffic_$lib.json $env $lib
  done
done
exit 0
