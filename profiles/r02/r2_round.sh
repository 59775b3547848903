# Round-2 checkpoint on the box: full GPU suite, then the profile round.
set -o pipefail
mkdir -p gpurun_out
export BMQCRC_GOLDEN_DIR=$PWD/tests/golden
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r2_gputests_round.log 2>&1; rc=$?
tail -3 gpurun_out/r2_gputests_round.log
[ $rc -eq 0 ] || exit $rc
bash tools/profile_round.sh ${1:-q1} 64k_x_64KiB 1M_x_256B zipf_4M 16_x_256MiB 1k_x_4KiB
