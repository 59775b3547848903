#!/bin/bash
# Same-box A/B of variants on the whole Zipf batch and two of its 1/8 shards
# (bench step ms), alternating builds, two rounds.
#   usage (on the box): tools/r3_ab_zipf.sh <tag> <variant|base> ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=$1; shift
L=blazingmq_amd/lib
mkdir -p gpurun_out
cp $L/libbmqcrc.so /tmp/abz_base.so
out=gpurun_out/${tag}.jsonl
rc=0
for rep in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then cp /tmp/abz_base.so $L/libbmqcrc.so; else cp $L/variant_$v.so $L/libbmqcrc.so; fi
    IFS=, read -ra ARGL <<< "${ZARGS:-,--shard 7/8,--shard 2/8}"
    for args in "${ARGL[@]}"; do
      timeout -k 10 200 python3 bench.py --config zipf_4M $args --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/${tag}_tmp.log 2>> gpurun_out/${tag}.err || { rc=1; break 3; }
      echo "{\"variant\": \"$v\", \"args\": \"$args\", \"rep\": $rep, \"bench\": $(tail -1 gpurun_out/${tag}_tmp.log)}" >> $out
    done
  done
done
cp /tmp/abz_base.so $L/libbmqcrc.so
python3 - "$out" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    b = d["bench"]
    print(d["variant"], d["args"] or "whole", d["rep"], b["ms_per_step"], b["roofline"]["kernel_avg_us"], b["parity"]["mismatches"])
PY
exit $rc
