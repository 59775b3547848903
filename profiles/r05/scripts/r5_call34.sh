#!/bin/bash
# round 5, GPU call 34: k_plan_map writes the long runs' head/tail entries
# and whole-group descriptors flattened over the wave, 64 items per store
# (product, BMQCRC_LONG_FLAT=1), against run by run (variant long0):
# parity + fuzz suites on the product, Zipf whole / 7/8 / 0/8 steps
# alternated, traced planner times, phase stamps of the product (pd3)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
VARIANTS="long0" PARITY=1 TAG=call34ab ROUNDS=3 STEPS=40 CONFIGS="zipf_4M zipf_4M:7/8 zipf_4M:0/8" \
  bash tools/r5_ab_multi.sh || exit $?
bash tools/plan_trace_ab.sh r5/call34pt "base long0 base long0" || exit $?
out=gpurun_out/r5/call34
mkdir -p $out
lib=blazingmq_amd/lib
cp $lib/libbmqcrc.so /tmp/base.so
cp $lib/variant_pd3.so $lib/libbmqcrc.so
for s in 7/8 0/8 0/1; do
  timeout -k 10 120 python3 tools/plan_trace_diag.py $s >> $out/stamps.jsonl 2>> $out/err.log \
    || { cp /tmp/base.so $lib/libbmqcrc.so; exit 1; }
done
cp /tmp/base.so $lib/libbmqcrc.so
cat $out/stamps.jsonl
