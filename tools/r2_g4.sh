set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 180 --timeout-method thread -k "speculative or shape_hint or whole_messages or 1M_x_256B or 64k_x_64KiB_full or small_ragged" > gpurun_out/r2_gputests4.log 2>&1; rc=$?
tail -12 gpurun_out/r2_gputests4.log
[ $rc -eq 0 ] || exit $rc
for c in 1M_x_256B 64k_x_64KiB 1k_x_4KiB; do
  timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline > gpurun_out/r2_bench4_$c.log 2>&1 || exit 1
  tail -1 gpurun_out/r2_bench4_$c.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["config"]["workload"][:12], d["value"], d["ms_per_step"], d["roofline"]["kernel_avg_us"], d["roofline"]["frac"], d["parity"])'
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r2p4_1M -o run --output-format csv -- python3 bench.py --config 1M_x_256B --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r2p4_1M.log 2>&1 || exit 1
find gpurun_out/r2p4_1M -name "*kernel_stats.csv" -exec cat {} \;
