#!/bin/bash
# A/B of several libraries in one box session: the parity tests of env 0 and 4 on every candidate
# (bitwise vs the oracle), the one-wave velocity micro-benchmark, then the interleaved bench A/B
# (tools/ab_bench.sh) for v0 at 4096 lanes and the 3-block config at 1024 lanes.
#   tools/ab_multi.sh base.so cand1.so [cand2.so ...]
set -uo pipefail
mkdir -p gpurun_out
( for i in $(seq 1 60); do date >> gpurun_out/heartbeat; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for lib in "${@:2}"; do
  T=tests/test_gpu.py
  MRP_LIB=$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
      "$T::test_step_parity_host_inputs[0]" "$T::test_step_parity_host_inputs[4]" "$T::test_device_autoreset_full_size[0]" \
      "$T::test_device_autoreset_full_size[4]" "$T::test_whole_episode_soak[0]" "$T::test_whole_episode_soak[4]" \
      > gpurun_out/ab_tests_$(basename $lib .so).log 2>&1 \
    || { echo "gpu tests failed for $lib"; tail -30 gpurun_out/ab_tests_$(basename $lib .so).log; exit 1; }
  echo "$lib: $(tail -1 gpurun_out/ab_tests_$(basename $lib .so).log)"
done
for lib in "$@"; do
  MRP_LIB=$lib timeout -k 10 120 python tools/velbench.py > gpurun_out/velbench_$(basename $lib .so).txt 2>&1 || { echo "velbench failed"; exit 1; }
  echo "== velbench $lib"; grep "blocks     1 " gpurun_out/velbench_$(basename $lib .so).txt
done
timeout -k 10 900 bash tools/ab_bench.sh "$@" || exit 1
ENV=4 LANES=1024 timeout -k 10 900 bash tools/ab_bench.sh "$@" || exit 1
exit 0
