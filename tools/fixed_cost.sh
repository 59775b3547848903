#!/bin/bash
# k_fold time vs batch size at 256 B per message: the intercept is the fixed
# per-launch cost (ramp-up + tail) that dominates the small-message config.
#   usage: tools/fixed_cost.sh [prefix] [msg counts] [extra bench flags]
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
prefix=${1:-fixed}
counts=${2:-"262144 524288 1048576 2097152 4194304"}
extra=${3:-}
: > gpurun_out/$prefix.jsonl
for n in $counts; do
    timeout -k 10 200 python bench.py --config 1M_x_256B --msgs $n --steps 50 --warmup 5 \
        --no-cpu-baseline --check 16 $extra > gpurun_out/${prefix}_$n.log 2>&1
    tail -1 gpurun_out/${prefix}_$n.log >> gpurun_out/$prefix.jsonl
    tail -1 gpurun_out/${prefix}_$n.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["config"]["n_msgs_total"], d["ms_per_step"], d["roofline"]["kernel_avg_us"])'
done
