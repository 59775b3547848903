#!/bin/bash
# Planner round: GPU suite on the product, parity + fuzz with the ragged
# planner replaced by the round-2 pair (variant_pair), phase stamps, and traced
# planner times on Zipf and its 1/8 shard.
#   usage (on the box): tools/r3_vec.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=$1
mkdir -p gpurun_out
L=blazingmq_amd/lib
T="python3 -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests -m gpu > gpurun_out/${tag}_gputests.log 2>&1 || { echo "gpu suite failed"; tail -20 gpurun_out/${tag}_gputests.log; exit 1; }
tail -1 gpurun_out/${tag}_gputests.log
if [ -f $L/variant_pair.so ]; then
  cp $L/libbmqcrc.so /tmp/vec_base.so
  cp $L/variant_pair.so $L/libbmqcrc.so
  timeout -k 10 400 $T tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -k "not map_given_up and not single_pass_planner" > gpurun_out/${tag}_sp_tests.log 2>&1
  rc=$?
  cp /tmp/vec_base.so $L/libbmqcrc.so
  tail -1 gpurun_out/${tag}_sp_tests.log
  [ $rc -eq 0 ] || { tail -20 gpurun_out/${tag}_sp_tests.log; exit 1; }
fi
timeout -k 10 300 tools/r3_stamps.sh gpurun_out/${tag}_stamps.jsonl pd3 pd3 > /dev/null || exit 1
for args in "--config zipf_4M" "--config zipf_4M --shard 7/8"; do
  t=$(echo "$args" | tr -c 'a-zA-Z0-9_\n' '_')
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_tr$t -o run --output-format csv -- \
      python3 bench.py $args --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${tag}_tr$t.log 2>&1 || exit 1
  grep -h "k_plan\|k_fold" gpurun_out/${tag}_tr$t/run_kernel_stats.csv | cut -d, -f1-4
done
