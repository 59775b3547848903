#!/bin/bash
# k_fold's fixed cost per launch: traced k_fold and planner times on Zipf
# shards 0/N for several N (time = S + W/N).
#   usage (on the box): tools/r3_fixed.sh <tag> [N ...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=$1; shift
mkdir -p gpurun_out
for n in ${*:-8 16 32 64 128}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_$n -o run --output-format csv -- \
      python3 bench.py --config zipf_4M --shard 0/$n --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/${tag}_$n.log 2>&1 || exit 1
  echo "N=$n step_ms=$(tail -1 gpurun_out/${tag}_$n.log | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')"
  grep -h "k_plan\|k_fold" gpurun_out/${tag}_$n/run_kernel_stats.csv | cut -d, -f1,2,4
done
