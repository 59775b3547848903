set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 180 --timeout-method thread -k "past_32_bits or leaves_current or 64k_x_64KiB_full or max_length" --durations=10 > gpurun_out/r2_gputests2.log 2>&1; rc=$?
tail -25 gpurun_out/r2_gputests2.log
exit $rc
