# Round-3: 4-byte seginfo entries.  GPU suite, planner traces (base vs r2),
# and a same-box A/B on Zipf, its 1/8 shard and 1k x 4 KiB.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export BMQCRC_GOLDEN_DIR=$PWD/tests/golden
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r3_seg4_gputests.log 2>&1; rc=$?
tail -3 gpurun_out/r3_seg4_gputests.log
[ $rc -eq 0 ] || exit $rc
bash tools/plan_trace_ab.sh pt6 "base r2" || exit $?
REPS=2 bash tools/ab_args.sh ab6 "base r2" "zipf:--config zipf_4M" \
  "shard:--config zipf_4M --shard 7/8" "1k:--config 1k_x_4KiB" "256:--config 1M_x_256B"
