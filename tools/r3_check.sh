# Round-3 checkpoint on the box: GPU suite, then one bench line per config.
set -o pipefail
mkdir -p gpurun_out
export BMQCRC_GOLDEN_DIR=$PWD/tests/golden
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r3_gputests.log 2>&1; rc=$?
tail -3 gpurun_out/r3_gputests.log
[ $rc -eq 0 ] || exit $rc
for c in ${*:-64k_x_64KiB 1M_x_256B}; do
    timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 5 > gpurun_out/r3_bench_$c.log 2>&1 || exit $?
    tail -1 gpurun_out/r3_bench_$c.log
done
