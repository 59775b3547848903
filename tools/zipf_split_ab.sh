#!/bin/bash
# zipf_split_time.py per library build (base = the product, others
# variant_<v>.so), the product restored after.
#   usage (GPU box): tools/zipf_split_ab.sh <out.jsonl> "<variants>" "<split args>" ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=$1; variants=$2; shift 2
lib=blazingmq_amd/lib
cp $lib/libbmqcrc.so /tmp/zsplit_base.so
rc=0
for v in $variants; do
  if [ "$v" = base ]; then cp /tmp/zsplit_base.so $lib/libbmqcrc.so; else cp $lib/variant_$v.so $lib/libbmqcrc.so; fi
  for a in "$@"; do
    timeout -k 10 300 python3 tools/zipf_split_time.py $a 2>/dev/null | sed "s/^{/{\"variant\": \"$v\", /" >> $out || { rc=$?; break 2; }
  done
done
cp /tmp/zsplit_base.so $lib/libbmqcrc.so
exit $rc
