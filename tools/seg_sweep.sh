#!/bin/bash
# Headline k_fold vs segment size and grid: the product build (automatic grid)
# and variant_bpc1 / variant_bpc2 (tools/build_variant.sh bpc1
# -DBMQCRC_TUNE_BITS=2, bpc2 -DBMQCRC_TUNE_BITS=8) forcing 1 or 2 blocks per CU.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
cfg=${1:-64k_x_64KiB}
lib=blazingmq_amd/lib
cp $lib/libbmqcrc.so /tmp/seg_sweep_base.so
for v in bpc1 bpc2; do
  cp $lib/variant_$v.so $lib/libbmqcrc.so
  for seg in 16384 32768 65536 131072; do
    timeout -k 10 200 python bench.py --config $cfg --seg-bytes $seg --steps 20 \
        --warmup 5 --no-cpu-baseline --check 32 > gpurun_out/sweep_${cfg}_${seg}_$v.log 2>&1
  done
done
cp /tmp/seg_sweep_base.so $lib/libbmqcrc.so
