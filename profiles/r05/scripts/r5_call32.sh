#!/bin/bash
# round 5, GPU call 32: the committed build as the driver runs it -- the GPU
# suite, the smoke, and bench.py with no flags
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r5/call32
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > $out/gpu_suite.log 2>&1 || { tail -20 $out/gpu_suite.log; exit 1; }
tail -1 $out/gpu_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -5 $out/smoke.log; exit 1; }
tail -2 $out/smoke.log
timeout -k 10 400 python bench.py > $out/bench_default.log 2>&1 || { tail -5 $out/bench_default.log; exit 1; }
grep '^{' $out/bench_default.log | cut -c1-400
