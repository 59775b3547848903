# Round-3: GPU suite on the product build (split tail), then planner block
# sizing: traces of Zipf and its 1/8 shard for base, pmt4, pmt8 and the 1/8
# shard's bench line per variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export BMQCRC_GOLDEN_DIR=$PWD/tests/golden
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r3_pmt_gputests.log 2>&1; rc=$?
tail -3 gpurun_out/r3_pmt_gputests.log
[ $rc -eq 0 ] || exit $rc
bash tools/plan_trace_ab.sh pt7 "base pmt4 pmt8" || exit $?
REPS=2 bash tools/ab_args.sh ab8 "base pmt4 pmt8" "shard:--config zipf_4M --shard 7/8" "zipf:--config zipf_4M"
