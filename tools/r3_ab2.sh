# Round-3 A/B 2: GPU suite on the product build (class-major single-pass
# planner with a grid-wide wait, right-aligned streams, one-line remainder
# skip), then same-box A/B against round 2 (r2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export BMQCRC_GOLDEN_DIR=$PWD/tests/golden
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r3_ab2_gputests.log 2>&1; rc=$?
tail -3 gpurun_out/r3_ab2_gputests.log
[ $rc -eq 0 ] || exit $rc
REPS=3 bash tools/ab_args.sh ab2 "base r2" \
  "256:--config 1M_x_256B" "64:--config 1M_x_256B --msg-bytes 64" \
  "128:--config 1M_x_256B --msg-bytes 128" "zipf:--config zipf_4M" \
  "shard:--config zipf_4M --shard 7/8"
