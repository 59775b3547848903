#!/bin/bash
# round 5, GPU call 18: the whole -m gpu suite and the smoke on the product
# build with the byte-granular remainder fold
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r5/call18
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    > $out/gpu_suite.log 2>&1 || { tail -30 $out/gpu_suite.log; exit 1; }
tail -3 $out/gpu_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { cat $out/smoke.log; exit 1; }
tail -3 $out/smoke.log
