#!/bin/bash
# Host cost per batch call, product against variants (tools/host_overhead.py).
#   usage (on the box): tools/r3_host.sh <out.jsonl> <variant|base> ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=$1; shift
L=blazingmq_amd/lib
mkdir -p gpurun_out
cp $L/libbmqcrc.so /tmp/host_base.so
rc=0
for rep in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then cp /tmp/host_base.so $L/libbmqcrc.so; else cp $L/variant_$v.so $L/libbmqcrc.so; fi
    for shape in "1000 4096" "64 256"; do
      echo -n "{\"variant\": \"$v\", \"res\": " >> $out
      timeout -k 10 120 python3 tools/host_overhead.py $shape 2000 >> $out 2>> gpurun_out/host.err || { rc=1; echo "null}" >> $out; break 3; }
      sed -i '$ s/$/}/' $out
    done
  done
done
cp /tmp/host_base.so $L/libbmqcrc.so
cat $out
exit $rc
