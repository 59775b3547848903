#!/bin/bash
# round 5, GPU call 27: raw per-wave stamps of the one-segment kernel
# (variant_fd1.so) for an analysis of where the end spread lies
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r5/call27
mkdir -p $out
lib=blazingmq_amd/lib
cp $lib/libbmqcrc.so /tmp/base.so
cp $lib/variant_fd1.so $lib/libbmqcrc.so
timeout -k 10 120 python3 tools/fold_trace_diag.py 1M_x_256B 1048576 256 $out/raw_1M_256.npy > $out/t.jsonl 2> $out/err.log || { cp /tmp/base.so $lib/libbmqcrc.so; exit 1; }
timeout -k 10 120 python3 tools/fold_trace_diag.py 1M_x_256B 2097152 128 $out/raw_2M_128.npy >> $out/t.jsonl 2>> $out/err.log || { cp /tmp/base.so $lib/libbmqcrc.so; exit 1; }
cp /tmp/base.so $lib/libbmqcrc.so
cat $out/t.jsonl
