# Round-3 A/B 3: GPU suite, planner kernel traces (Zipf and its 1/8 shard)
# for the product build vs round 2, then bench A/B of the stream geometry.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export BMQCRC_GOLDEN_DIR=$PWD/tests/golden
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r3_ab3_gputests.log 2>&1; rc=$?
tail -3 gpurun_out/r3_ab3_gputests.log
[ $rc -eq 0 ] || exit $rc
bash tools/plan_trace_ab.sh pt3 "base r2 oldplan" || exit $?
REPS=2 bash tools/ab_args.sh ab3 "base r2 ra1 nora oldplan" \
  "256:--config 1M_x_256B" "64:--config 1M_x_256B --msg-bytes 64" \
  "128:--config 1M_x_256B --msg-bytes 128" "zipf:--config zipf_4M"
