set -o pipefail
tools/ab_swap.sh r2ab_loop old 1M_x_256B zipf_4M 64k_x_64KiB 1k_x_4KiB > gpurun_out/r2ab_loop.log 2>&1; rc=$?
grep -v "^==" gpurun_out/r2ab_loop.log | tail -20
exit $rc
