# Round-3 A/B 1: GPU suite on the product build, then same-box A/B of the
# single-pass planner + right-aligned streams (base) against round 2 (r2), the
# round-2 planner pair (oldplan), and narrower right alignment (ra0, ra2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export BMQCRC_GOLDEN_DIR=$PWD/tests/golden
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r3_ab1_gputests.log 2>&1; rc=$?
tail -3 gpurun_out/r3_ab1_gputests.log
[ $rc -eq 0 ] || exit $rc
REPS=2 bash tools/ab_args.sh ab1 "base r2 oldplan ra0 ra2" \
  "256:--config 1M_x_256B" "64:--config 1M_x_256B --msg-bytes 64" \
  "128:--config 1M_x_256B --msg-bytes 128" "zipf:--config zipf_4M" \
  "shard:--config zipf_4M --shard 7/8" "head:--config 64k_x_64KiB"
