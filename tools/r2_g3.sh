set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread --deselect "tests/test_gpu_parity.py::test_segment_count_past_32_bits" > gpurun_out/r2_gputests3.log 2>&1; rc=$?
tail -5 gpurun_out/r2_gputests3.log
[ $rc -eq 0 ] || exit $rc
for c in 64k_x_64KiB 1M_x_256B zipf_4M 16_x_256MiB 1k_x_4KiB; do
  timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline > gpurun_out/r2_bench3_$c.log 2>&1 || exit 1
  tail -1 gpurun_out/r2_bench3_$c.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["config"]["workload"][:12], d["value"], d["ms_per_step"], d["roofline"]["kernel_avg_us"], d["roofline"]["frac"], d["parity"])'
done
