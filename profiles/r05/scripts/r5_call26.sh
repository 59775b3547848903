#!/bin/bash
# round 5, GPU call 26: per-wave phase stamps of the one-segment kernel on
# small-message batches (diagnostic build variant_fd1.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r5/call26
mkdir -p $out
lib=blazingmq_amd/lib
cp $lib/libbmqcrc.so /tmp/base.so
cp $lib/variant_fd1.so $lib/libbmqcrc.so
for w in "1M_x_256B" "1M_x_256B 4194304 256" "1M_x_256B 2097152 128" "1M_x_256B 4194304 64"; do
  timeout -k 10 120 python3 tools/fold_trace_diag.py $w >> $out/fold_trace_one.jsonl 2> $out/err.log || { cp /tmp/base.so $lib/libbmqcrc.so; exit 1; }
done
cp /tmp/base.so $lib/libbmqcrc.so
cat $out/fold_trace_one.jsonl
