#!/bin/bash
# k_plan_map per-block phase stamps (8 per block, tools/plan_trace_diag.py):
# variant_pd3.so on the whole Zipf batch, variant_pd3s.so (TUNE bit 9: the
# single-pass planner on single-tile blocks too) on its 1/8 shard.
#   usage (on the box): tools/r3_stamps.sh <out.jsonl> [variant-for-whole variant-for-shard]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
out=$1; vw=${2:-pd3}; vs=${3:-pd3s}
L=blazingmq_amd/lib
cp $L/libbmqcrc.so /tmp/stamps_base.so
rc=0
for pair in "$vw 0/1" "$vs 7/8" "$vw 0/1" "$vs 7/8"; do
  set -- $pair
  cp $L/variant_$1.so $L/libbmqcrc.so
  echo "{\"variant\": \"$1\"}" >> $out
  timeout -k 10 120 python3 tools/plan_trace_diag.py $2 >> $out 2>> gpurun_out/stamps.err || { rc=$?; break; }
done
cp /tmp/stamps_base.so $L/libbmqcrc.so
cat $out
exit $rc
