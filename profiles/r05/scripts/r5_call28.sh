#!/bin/bash
# round 5, GPU call 28: the one-segment kernel with block claims (variant
# oneclaims) against the static grid-stride product, plus the per-wave end
# spread with claims (variant fdc: claims + stamps) and with the progress
# priority (variants oneprio, fdp)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r5/call28
mkdir -p $out
lib=blazingmq_amd/lib
cp $lib/libbmqcrc.so /tmp/base.so
cp $lib/variant_fdc.so $lib/libbmqcrc.so
timeout -k 10 120 python3 tools/fold_trace_diag.py 1M_x_256B 1048576 256 $out/raw_c_1M_256.npy > $out/t.jsonl 2> $out/err.log || { cp /tmp/base.so $lib/libbmqcrc.so; exit 1; }
timeout -k 10 120 python3 tools/fold_trace_diag.py 1M_x_256B 2097152 128 $out/raw_c_2M_128.npy >> $out/t.jsonl 2>> $out/err.log || { cp /tmp/base.so $lib/libbmqcrc.so; exit 1; }
cp $lib/variant_fdp.so $lib/libbmqcrc.so
timeout -k 10 120 python3 tools/fold_trace_diag.py 1M_x_256B 1048576 256 $out/raw_p_1M_256.npy >> $out/t.jsonl 2>> $out/err.log || { cp /tmp/base.so $lib/libbmqcrc.so; exit 1; }
timeout -k 10 120 python3 tools/fold_trace_diag.py 1M_x_256B 2097152 128 $out/raw_p_2M_128.npy >> $out/t.jsonl 2>> $out/err.log || { cp /tmp/base.so $lib/libbmqcrc.so; exit 1; }
cp /tmp/base.so $lib/libbmqcrc.so
cat $out/t.jsonl
VARIANTS="oneclaims oneprio" PARITY=0 PARITY_VARIANTS="oneclaims oneprio" TAG=call28ab \
  CONFIGS="1048576:256:4 4194304:256:4 2097152:128:4 4194304:64:4 1048576:200:4 64k_x_64KiB" \
  bash tools/r5_ab_multi.sh
