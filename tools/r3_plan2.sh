# Round-3 planner checkpoint: GPU suite on the product build, per-block
# phase stamps (pd3 / pd4 diagnostic builds), planner kernel traces (base vs
# round 2) on Zipf 4M and its 1/8 shard.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export BMQCRC_GOLDEN_DIR=$PWD/tests/golden
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r3_plan2_gputests.log 2>&1; rc=$?
tail -3 gpurun_out/r3_plan2_gputests.log
[ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/pd3.jsonl
bash tools/r3_pd3.sh || exit $?
bash tools/plan_trace_ab.sh pt5 "base r2"
REPS=2 bash tools/ab_args.sh ab5 "base split r2" \
  "256:--config 1M_x_256B" "64:--config 1M_x_256B --msg-bytes 64" \
  "128:--config 1M_x_256B --msg-bytes 128"
