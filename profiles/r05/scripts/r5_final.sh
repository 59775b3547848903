#!/bin/bash
# round 5, final-build evidence (one GPU call): per-config bench lines,
# kernel traces and FETCH/WRITE passes (tools/profile_round.sh r5f), the
# HBM-resident small messages under rocprofv3 (4 rotating copies), the
# strong-scaling shard forecast, the smoke
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/${P:-r5f}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/${P:-r5f}/gpu_suite.log 2>&1 || { tail -20 gpurun_out/${P:-r5f}/gpu_suite.log; exit 1; }
tail -1 gpurun_out/${P:-r5f}/gpu_suite.log
timeout -k 10 1500 bash tools/profile_round.sh ${P:-r5f} 64k_x_64KiB 1M_x_256B 16_x_256MiB zipf_4M 1k_x_4KiB \
    > gpurun_out/${P:-r5f}/profile_round.log 2>&1 || { tail -5 gpurun_out/${P:-r5f}/profile_round.log; exit 1; }
grep -h '^{' gpurun_out/bench_${P:-r5f}_*.log | cut -c1-160
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for w in "1048576 256" "2097152 256" "4194304 256" "2097152 128" "4194304 64" "1048576 200"; do
  set -- $w
  tag=rot_$1_$2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${P:-r5f}/prof_$tag -o run --output-format csv \
      -- python3 bench.py --config 1M_x_256B --msgs $1 --msg-bytes $2 --rotate 4 --steps 30 --warmup 5 \
      --no-cpu-baseline > gpurun_out/${P:-r5f}/prof_$tag.log 2>&1 || exit $?
  tail -1 gpurun_out/${P:-r5f}/prof_$tag.log | cut -c1-200
done
timeout -k 10 900 bash tools/shard_forecast.sh sf_${P:-r5f} 8 4 > gpurun_out/${P:-r5f}/shard_forecast.log 2>&1 || exit $?
tail -16 gpurun_out/${P:-r5f}/shard_forecast.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${P:-r5f}/smoke.log 2>&1
