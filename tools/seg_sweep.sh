#!/bin/bash
# Headline k_fold vs segment size and grid (1 or 2 blocks per CU).
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
cfg=${1:-64k_x_64KiB}
for seg in 16384 32768 65536 131072; do
  for t in 0 2; do
    BMQCRC_TUNE=$t timeout -k 10 200 python bench.py --config $cfg --seg-bytes $seg --steps 20 \
        --warmup 5 --no-cpu-baseline --check 32 > gpurun_out/sweep_${cfg}_${seg}_t$t.log 2>&1
  done
done
