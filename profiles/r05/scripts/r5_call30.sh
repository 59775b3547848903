#!/bin/bash
# round 5, GPU call 30: k_plan_map's per-block phase stamps on Zipf's 7/8
# shard and the whole batch, with component skips (diagnostic builds: pd3
# stamps only, pd4 no seginfo stores, ps1 no histogram atomics, ps2 no
# last-segment claims, ps4 no full-run writes, ps8 no last-segment stores)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r5/call30
mkdir -p $out
lib=blazingmq_amd/lib
cp $lib/libbmqcrc.so /tmp/base.so
for r in 1 2; do
for v in pd3 pd4 ps1 ps2 ps4 ps8; do
  cp $lib/variant_$v.so $lib/libbmqcrc.so
  for s in 7/8 0/1; do
    echo "{\"variant\": \"$v\", \"round\": $r}" >> $out/stamps.jsonl
    timeout -k 10 120 python3 tools/plan_trace_diag.py $s >> $out/stamps.jsonl 2>> $out/err.log \
      || { cp /tmp/base.so $lib/libbmqcrc.so; tail -5 $out/err.log; exit 1; }
  done
done
done
cp /tmp/base.so $lib/libbmqcrc.so
cat $out/stamps.jsonl
