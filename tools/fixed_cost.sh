#!/bin/bash
# k_fold time vs batch size at 256 B per message: the intercept is the fixed
# per-launch cost (ramp-up + tail) that dominates the small-message config.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for n in 262144 524288 1048576 2097152 4194304; do
    timeout -k 10 200 python bench.py --config 1M_x_256B --msgs $n --steps 20 --warmup 5 \
        --no-cpu-baseline --check 16 > gpurun_out/fixed_$n.log 2>&1
done
