# Round-3 planner check on the box: GPU suite on the product build, then
# planner/fold kernel traces (Zipf 4M and its 1/8 shard) for the product
# build and the round-2 planner pair (variant_oldplan, TUNE bit7), alternated.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export BMQCRC_GOLDEN_DIR=$PWD/tests/golden
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r3_plan_gputests.log 2>&1; rc=$?
tail -3 gpurun_out/r3_plan_gputests.log
[ $rc -eq 0 ] || exit $rc
bash tools/plan_trace_ab.sh ${1:-pm1} "base oldplan base oldplan"
