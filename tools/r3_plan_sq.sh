#!/bin/bash
# SQ counters of the planner kernels (k_plan_map on the Zipf batch, the pair
# on its 1/8 shard): two --pmc passes per case, 8 SQ counters each.
# usage (on the box): tools/r3_plan_sq.sh <prefix>
set -eo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
prefix=$1
mkdir -p gpurun_out
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS"
for args in "--config zipf_4M" "--config zipf_4M --shard 7/8"; do
    tag=$(echo "$args" | tr -c 'a-zA-Z0-9_\n' '_')
    for p in 1 2; do
        eval c=\$P$p
        echo "== $tag pass $p $(date +%T)"
        timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/${prefix}_${tag}_p$p -o run --output-format csv -- \
            python3 bench.py $args --steps 3 --warmup 1 --no-cpu-baseline \
            --settle-seconds 0 --no-kernel-timing > gpurun_out/${prefix}_${tag}_p$p.log 2>&1
    done
done
