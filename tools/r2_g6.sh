set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread --deselect "tests/test_gpu_parity.py::test_segment_count_past_32_bits" > gpurun_out/r2_gputests6.log 2>&1; rc=$?
tail -2 gpurun_out/r2_gputests6.log
[ $rc -eq 0 ] || exit $rc
: > gpurun_out/r2_shards.jsonl
timeout -k 10 200 python3 bench.py --config zipf_4M --no-cpu-baseline >> gpurun_out/r2_shards.jsonl 2>/dev/null || exit 1
for sh in 0/8 3/8 7/8 0/4 3/4; do
  timeout -k 10 200 python3 bench.py --config zipf_4M --shard $sh --no-cpu-baseline >> gpurun_out/r2_shards.jsonl 2>/dev/null || exit 1
done
python3 - <<'PY'
import json
for l in open('gpurun_out/r2_shards.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print(d['config']['workload'][:60], d['ms_per_step'], d['roofline']['kernel_avg_us'], d['roofline']['frac'])
PY
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r2p6_s78 -o run --output-format csv -- python3 bench.py --config zipf_4M --shard 7/8 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r2p6_s78.log 2>&1 || exit 1
find gpurun_out/r2p6_s78 -name "*kernel_stats.csv" -exec cat {} \;
