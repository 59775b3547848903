#!/bin/bash
# Per-wave k_fold stamps (tools/fold_trace_diag.py) with the FOLD_DIAG
# variant swapped in, the product restored after.
#   usage (GPU box): [V=<variant, default fd1>] tools/fold_trace_run.sh <out dir> "<diag args>" ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=$1; shift
mkdir -p "$out"
lib=blazingmq_amd/lib
cp $lib/libbmqcrc.so /tmp/fold_trace_base.so
cp $lib/variant_${V:-fd1}.so $lib/libbmqcrc.so
rc=0; i=0
for spec in "$@"; do
  i=$((i + 1))
  timeout -k 10 120 python3 tools/fold_trace_diag.py $spec $out/raw_$i.npy > $out/trace_$i.txt 2>&1 || { rc=$?; break; }
done
cp /tmp/fold_trace_base.so $lib/libbmqcrc.so
exit $rc
