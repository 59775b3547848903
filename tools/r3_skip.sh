#!/bin/bash
# k_plan_map phase stamps of component-skip diagnostic builds on the whole
# Zipf batch (variant_<v>.so built with -DBMQCRC_PLAN_DIAG=3
# -DBMQCRC_PLAN_SKIP=...; the map is voided, CRCs stay exact).
#   usage (on the box): tools/r3_skip.sh <out.jsonl> <variant> ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
out=$1; shift
L=blazingmq_amd/lib
cp $L/libbmqcrc.so /tmp/skip_base.so
rc=0
for rep in 1 2; do
  for v in "$@"; do
    cp $L/variant_$v.so $L/libbmqcrc.so
    echo "{\"variant\": \"$v\"}" >> $out
    timeout -k 10 120 python3 tools/plan_trace_diag.py 0/1 >> $out 2>> gpurun_out/skip.err || { rc=$?; break 2; }
  done
done
cp /tmp/skip_base.so $L/libbmqcrc.so
exit $rc
