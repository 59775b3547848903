set -o pipefail
mkdir -p gpurun_out/tail
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "many_rows or speculative or one_segment or config or shape_hint" > gpurun_out/tail/tests.log 2>&1 && \
REPS=2 timeout -k 10 700 bash tools/ab_args.sh tail/ab "base notail head" "256:--config 1M_x_256B" "4M256:--config 1M_x_256B --msgs 4194304" "128:--config 1M_x_256B --msgs 2097152 --msg-bytes 128" "64:--config 1M_x_256B --msgs 4194304 --msg-bytes 64" "200:--config 1M_x_256B --msg-bytes 200" "hl:--config 64k_x_64KiB" > gpurun_out/tail/ab.log 2>&1
rc=$?
tail -3 gpurun_out/tail/tests.log
cat gpurun_out/tail/ab.log
exit $rc
