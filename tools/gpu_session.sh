set -uo pipefail
mkdir -p gpurun_out
( for i in $(seq 1 40); do date >> gpurun_out/heartbeat; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_drv.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_drv.log; exit 1; }
tail -1 gpurun_out/bench_drv.log
MRP_LIB=gym_puzzles_amd/libmrp_stamps.so timeout -k 10 120 python tools/lane_replay.py 0 4096 8 8 > gpurun_out/replay_w8.txt 2>&1 || { echo "replay failed"; tail gpurun_out/replay_w8.txt; exit 1; }
cat gpurun_out/replay_w8.txt
