#!/bin/bash
# Per-block k_plan_map stamps (tools/plan_trace_diag.py) with a PLAN_DIAG
# variant swapped in (default pd3), the product restored after.
#   usage (GPU box): [V=<variant>] tools/plan_trace_run.sh <out dir> <shard i/N> ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=$1; shift
mkdir -p "$out"
lib=blazingmq_amd/lib
cp $lib/libbmqcrc.so /tmp/plan_trace_base.so
cp $lib/variant_${V:-pd3}.so $lib/libbmqcrc.so
rc=0
for sh in "$@"; do
  timeout -k 10 120 python3 tools/plan_trace_diag.py $sh >> $out/trace.jsonl 2>> $out/trace.err || { rc=$?; break; }
done
cp /tmp/plan_trace_base.so $lib/libbmqcrc.so
exit $rc
