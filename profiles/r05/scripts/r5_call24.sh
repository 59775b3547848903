#!/bin/bash
# round 5, GPU call 24: per-wave phase stamps of k_fold on small batches
# (diagnostic build variant_fd1.so), to see where a launch-bound step goes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r5/call24
mkdir -p $out
lib=blazingmq_amd/lib
cp $lib/libbmqcrc.so /tmp/base.so
cp $lib/variant_fd1.so $lib/libbmqcrc.so
for w in "1k_x_4KiB" "1M_x_256B 4096 1024" "1M_x_256B 20000 256" "1M_x_256B 1000 16384"; do
  timeout -k 10 120 python3 tools/fold_trace_diag.py $w >> $out/fold_trace_small.jsonl 2> $out/err.log || { cp /tmp/base.so $lib/libbmqcrc.so; exit 1; }
done
cp /tmp/base.so $lib/libbmqcrc.so
cat $out/fold_trace_small.jsonl
