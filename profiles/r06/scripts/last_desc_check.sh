#!/bin/bash
# One GPU call for the planner's last-segment descriptors (BMQCRC_LAST_DESC):
# the GPU suite, traced planner/fold times base vs nold (Zipf and its 1/8
# shard, two alternations), and FETCH/WRITE passes of the Zipf batch per build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/ld
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/suite.log 2>&1 || { tail -30 $O/suite.log; exit 1; }
tail -1 $O/suite.log
timeout -k 10 900 bash tools/plan_trace_ab.sh ld/pt "base nold base nold" > $O/pt.log 2>&1 || { tail -5 $O/pt.log; exit 1; }
timeout -k 10 200 bash tools/pmc_variant_pass.sh $O/pmc_base base --config zipf_4M > /dev/null || exit 1
timeout -k 10 200 bash tools/pmc_variant_pass.sh $O/pmc_nold nold --config zipf_4M > /dev/null || exit 1
echo done
