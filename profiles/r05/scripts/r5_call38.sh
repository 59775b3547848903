#!/bin/bash
# round 5, GPU call 38: raw per-wave k_fold stamps (variant fd1) of Zipf's
# 7/8 shard and the whole batch, for the end-spread analysis
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r5/call38
mkdir -p $out
lib=blazingmq_amd/lib
cp $lib/libbmqcrc.so /tmp/base.so
cp $lib/variant_fd1.so $lib/libbmqcrc.so
timeout -k 10 180 python3 tools/fold_trace_diag.py zipf_4M:7/8 0 0 $out/raw_shard78.npy >> $out/fold_trace.jsonl 2>> $out/err.log \
  && timeout -k 10 180 python3 tools/fold_trace_diag.py zipf_4M 0 0 $out/raw_whole.npy >> $out/fold_trace.jsonl 2>> $out/err.log
rc=$?
cp /tmp/base.so $lib/libbmqcrc.so
exit $rc
