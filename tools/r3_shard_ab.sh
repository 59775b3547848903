#!/bin/bash
# Same-box A/B of planner variants on Zipf shards: bench step time (ms) of
# shard 7/8 and 0/8 per variant, then a traced run of each.
#   usage (on the box): tools/r3_shard_ab.sh <tag> <variant|base> ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=$1; shift
L=blazingmq_amd/lib
mkdir -p gpurun_out
cp $L/libbmqcrc.so /tmp/shab_base.so
out=gpurun_out/${tag}.jsonl
rc=0
for rep in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then cp /tmp/shab_base.so $L/libbmqcrc.so; else cp $L/variant_$v.so $L/libbmqcrc.so; fi
    for sh in 7/8 0/8; do
      timeout -k 10 200 python3 bench.py --config zipf_4M --shard $sh --no-cpu-baseline --steps 30 --warmup 5 > gpurun_out/${tag}_tmp.log 2>> gpurun_out/${tag}.err || { rc=1; break 3; }
      echo "{\"variant\": \"$v\", \"shard\": \"$sh\", \"rep\": $rep, \"bench\": $(tail -1 gpurun_out/${tag}_tmp.log)}" >> $out
    done
  done
done
for v in "$@"; do
  [ $rc -eq 0 ] || break
  if [ "$v" = base ]; then cp /tmp/shab_base.so $L/libbmqcrc.so; else cp $L/variant_$v.so $L/libbmqcrc.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_tr_$v -o run --output-format csv -- \
      python3 bench.py --config zipf_4M --shard 7/8 --no-cpu-baseline --steps 20 --warmup 3 > /dev/null 2>&1 || rc=1
done
cp /tmp/shab_base.so $L/libbmqcrc.so
python3 - "$out" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d["variant"], d["shard"], d["rep"], d["bench"]["ms_per_step"], d["bench"]["parity"])
PY
exit $rc
