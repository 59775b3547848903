#!/bin/bash
# round 5, GPU call 33: k_plan_map phase stamps on Zipf and its 7/8 shard
# with finer full-run skips (diagnostic builds: pd3 stamps only, psl no
# long-run writes, pss no short-run writes, psn full-run slots mapped but
# not stored)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r5/call33
mkdir -p $out
lib=blazingmq_amd/lib
cp $lib/libbmqcrc.so /tmp/base.so
for r in 1 2; do
for v in pd3 psl pss psn; do
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
