#!/bin/bash
# Same-box A/B of the planner kernels of two library builds (product vs
# variant_<name>.so): rocprofv3 kernel trace of Zipf (whole batch and one 1/8
# shard) per build, then the per-kernel averages.
#   usage (on the box): tools/plan_ab.sh <prefix> <variant>
set -eo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
prefix=$1; name=$2
lib=blazingmq_amd/lib
cp $lib/libbmqcrc.so /tmp/plan_ab_base.so
for rep in 1 2; do
  for v in base $name; do
    if [ $v = base ]; then cp /tmp/plan_ab_base.so $lib/libbmqcrc.so; else cp $lib/variant_$v.so $lib/libbmqcrc.so; fi
    for args in "" "--shard 7/8"; do
      tag=${prefix}_${v}_${rep}_$(echo "$args" | tr -d ' /-')
      timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/$tag -o run --output-format csv -- \
          python3 bench.py --config zipf_4M --steps 10 --warmup 2 --no-cpu-baseline --settle-seconds 0.5 $args \
          > gpurun_out/$tag.log 2>&1 || { cp /tmp/plan_ab_base.so $lib/libbmqcrc.so; exit 3; }
      echo "$v rep$rep [$args] $(tail -1 gpurun_out/$tag.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d["parity"]["mismatches"])') $(grep -h 'k_plan\|k_fold' gpurun_out/$tag/run_kernel_stats.csv | awk -F, '{printf "%s=%.1f ", $1, $4/1000}')"
    done
  done
done
cp /tmp/plan_ab_base.so $lib/libbmqcrc.so
