#!/bin/bash
# SQ wave-cycle breakdown of k_fold per bench config (one --pmc pass each).
# usage (on the box): [COUNTERS="..."] tools/sq_counters.sh <prefix> [config ...]
set -eo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
prefix=$1
shift
configs=${*:-"1M_x_256B zipf_4M 64k_x_64KiB"}
# at most 8 SQ counters per pass (MI355X_MICROARCH.md, rocprofv3 PMC slots)
COUNTERS=${COUNTERS:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES"}
mkdir -p gpurun_out
for c in $configs; do
    echo "== $c $(date +%T)"
    timeout -k 10 300 rocprofv3 --pmc $COUNTERS --kernel-trace -d gpurun_out/${prefix}_$c -o run --output-format csv -- \
        python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline \
        --settle-seconds 0 --no-kernel-timing > gpurun_out/${prefix}_$c.log 2>&1
done
