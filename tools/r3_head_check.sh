#!/bin/bash
# Round-end check of the committed build on the box: the GPU suite, smoke(),
# the default bench line and its rocprofv3 kernel trace.  GPU box only.
#   usage: tools/r3_head_check.sh <prefix>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
p=${1:-hc}
mkdir -p gpurun_out/$p
export BMQCRC_GOLDEN_DIR=$PWD/tests/golden
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread \
    > gpurun_out/$p/gputests.log 2>&1 || { tail -20 gpurun_out/$p/gputests.log; exit 1; }
tail -1 gpurun_out/$p/gputests.log
timeout -k 10 180 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/$p/smoke.log 2>&1 || { tail -5 gpurun_out/$p/smoke.log; exit 1; }
tail -1 gpurun_out/$p/smoke.log
timeout -k 10 240 python bench.py > gpurun_out/$p/bench.log 2>&1 || { tail -5 gpurun_out/$p/bench.log; exit 1; }
tail -1 gpurun_out/$p/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/$p/prof" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/$p/prof.log" 2>&1 || exit 1
find "$GRAFT_REPO_ROOT/gpurun_out/$p/prof" -name "*kernel_stats.csv" -exec head -5 {} \;
