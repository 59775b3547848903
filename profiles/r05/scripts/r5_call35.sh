#!/bin/bash
# round 5, GPU call 35: evidence for the final build (flattened long-run
# planner writes): the GPU suite, the smoke, Zipf's bench line + kernel
# trace + FETCH/WRITE passes, and the shard forecast
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r5l
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > $out/gpu_suite.log 2>&1 || { tail -20 $out/gpu_suite.log; exit 1; }
tail -1 $out/gpu_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -5 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 600 bash tools/profile_round.sh r5l zipf_4M > $out/profile_round.log 2>&1 || { tail -5 $out/profile_round.log; exit 1; }
grep -h '^{' gpurun_out/bench_r5l_*.log | cut -c1-200
timeout -k 10 800 bash tools/shard_forecast.sh sf_r5l 8 4 > $out/shard_forecast.log 2>&1 || exit $?
tail -16 $out/shard_forecast.log
