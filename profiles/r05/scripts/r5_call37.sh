#!/bin/bash
# round 5, GPU call 37: per-wave k_fold stamps of the final build (variant
# fd1, BMQCRC_FOLD_DIAG=1) on Zipf, its 7/8 shard, and 4M x 256 B: where the
# start and the drain go
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r5/call37
mkdir -p $out
lib=blazingmq_amd/lib
cp $lib/libbmqcrc.so /tmp/base.so
cp $lib/variant_fd1.so $lib/libbmqcrc.so
for c in "zipf_4M:7/8" "zipf_4M:0/8" "zipf_4M" "1M_x_256B 4194304 256"; do
  timeout -k 10 180 python3 tools/fold_trace_diag.py $c >> $out/fold_trace.jsonl 2>> $out/err.log \
    || { cp /tmp/base.so $lib/libbmqcrc.so; tail -5 $out/err.log; exit 1; }
done
cp /tmp/base.so $lib/libbmqcrc.so
cat $out/fold_trace.jsonl
