#!/bin/bash
# bmqcrc_opts.max_len (ABI 2.4) on the box: its GPU test, the speculative /
# planned / declared parity tests around it, then bench lines with the
# declared-bound leg for the small-message config, the headline and
# configs[0].  GPU box only.
#   usage: tools/r3_declared.sh <prefix>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
p=${1:-dl}
mkdir -p gpurun_out/$p
export BMQCRC_GOLDEN_DIR=$PWD/tests/golden
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 \
    --timeout-method thread -k "declared or speculative or config_1k" > gpurun_out/$p/tests.log 2>&1 \
    || { tail -30 gpurun_out/$p/tests.log; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/$p/tests.log
for c in 1M_x_256B 64k_x_64KiB 1k_x_4KiB; do
    steps=100; [ $c = 1k_x_4KiB ] && steps=400
    timeout -k 10 240 python3 bench.py --config $c --steps $steps --warmup 10 --no-cpu-baseline \
        > gpurun_out/$p/bench_$c.log 2>&1 || { tail -5 gpurun_out/$p/bench_$c.log; exit 1; }
    tail -1 gpurun_out/$p/bench_$c.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["config"]["workload"][:12], d["value"], d["ms_per_step"], d["planned_ms_per_step"], d["declared_ms_per_step"], d["declared_kernels_per_step"], d["parity"])'
done
