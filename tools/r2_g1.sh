set -o pipefail
mkdir -p gpurun_out
export BMQCRC_GOLDEN_DIR=$PWD/tests/golden
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r2_gputests1.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r2_gputests1.log; exit 1; }
tail -3 gpurun_out/r2_gputests1.log
timeout -k 10 120 tests/cpp/bin/bmqp_selftest gpu > gpurun_out/r2_selftest_gpu.log 2>&1 && tail -1 gpurun_out/r2_selftest_gpu.log
BENCH_DEVICE=0 timeout -k 10 300 python3 bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/r2_rehearsal_n2.log 2>&1; echo "rehearsal rc=$?"; tail -1 gpurun_out/r2_rehearsal_n2.log
timeout -k 10 300 python3 bench.py --protocol > gpurun_out/r2_protocol.log 2>&1; echo "protocol rc=$?"; tail -4 gpurun_out/r2_protocol.log
