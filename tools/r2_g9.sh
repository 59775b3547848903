set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread --deselect "tests/test_gpu_parity.py::test_segment_count_past_32_bits" > gpurun_out/r2_gputests9.log 2>&1; rc=$?
tail -2 gpurun_out/r2_gputests9.log
[ $rc -eq 0 ] || exit $rc
: > gpurun_out/r2_shards2.jsonl
for args in "--config zipf_4M" "--config zipf_4M --shard 7/8" "--config zipf_4M --shard 0/8" "--config zipf_4M --shard 3/4" "--config 64k_x_64KiB --msg-bytes 8192" "--config 64k_x_64KiB --msg-bytes 4096" "--config 1M_x_256B" "--config 16_x_256MiB"; do
  timeout -k 10 200 python3 bench.py $args --no-cpu-baseline --check 64 > gpurun_out/r2_s2.log 2>&1 || exit 1
  tail -1 gpurun_out/r2_s2.log >> gpurun_out/r2_shards2.jsonl
  tail -1 gpurun_out/r2_s2.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('$args', d['ms_per_step'], d['roofline']['kernel_avg_us'], d['roofline']['frac'], d['parity'])"
done
