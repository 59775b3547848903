set -o pipefail
mkdir -p gpurun_out/rot
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "speculative or one_segment" > gpurun_out/rot/tests.log 2>&1 && \
cp blazingmq_amd/lib/libbmqcrc.so /tmp/rot_base.so && cp blazingmq_amd/lib/variant_rot.so blazingmq_amd/lib/libbmqcrc.so && \
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "speculative or one_segment" > gpurun_out/rot/tests_rot.log 2>&1; rc=$?
cp /tmp/rot_base.so blazingmq_amd/lib/libbmqcrc.so
[ $rc -eq 0 ] && REPS=2 timeout -k 10 600 bash tools/ab_args.sh rot/ab "base rot" "256:--config 1M_x_256B" "4M256:--config 1M_x_256B --msgs 4194304" "128:--config 1M_x_256B --msgs 2097152 --msg-bytes 128" "64:--config 1M_x_256B --msgs 4194304 --msg-bytes 64" "hl:--config 64k_x_64KiB" > gpurun_out/rot/ab.log 2>&1 && \
V=fdrot timeout -k 10 300 bash tools/fold_trace_run.sh gpurun_out/rot/ft "1M_x_256B 1048576 256" "1M_x_256B 4194304 256"
rc=$?
tail -2 gpurun_out/rot/tests.log gpurun_out/rot/tests_rot.log
cat gpurun_out/rot/ab.log
exit $rc
