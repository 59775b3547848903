#!/bin/bash
# A round's final-build evidence in one GPU call (on the box):
#   1. the GPU suite;  2. tools/profile_round.sh <P> over the five BASELINE
#   configs (bench line, rocprofv3 kernel trace, FETCH_SIZE / WRITE_SIZE
#   passes);  3. HBM-resident small messages (4 rotating copies) under
#   rocprofv3 --kernel-trace --stats;  4. SQ counter passes on them
#   (tools/sq_small.sh);  5. the strong-scaling shard forecast
#   (tools/shard_forecast.sh, 8 and 4);  6. the smoke.
# Every GPU step has its own time limit; the first failure ends the call.
#   usage: P=<prefix> tools/round_final.sh      (outputs: gpurun_out/<P>/...)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
P=${P:-rNf}
O=gpurun_out/$P
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    --junitxml=$O/gpu_suite.xml > $O/gpu_suite.log 2>&1 || { tail -20 $O/gpu_suite.log; exit 1; }
tail -1 $O/gpu_suite.log
timeout -k 10 1500 bash tools/profile_round.sh $P 64k_x_64KiB 1M_x_256B 16_x_256MiB zipf_4M 1k_x_4KiB \
    > $O/profile_round.log 2>&1 || { tail -5 $O/profile_round.log; exit 1; }
grep -h '^{' gpurun_out/bench_${P}_*.log | cut -c1-160
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for w in "1048576 256" "2097152 256" "4194304 256" "2097152 128" "4194304 64" "1048576 200"; do
  set -- $w
  tag=rot_$1_$2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$tag -o run --output-format csv \
      -- python3 bench.py --config 1M_x_256B --msgs $1 --msg-bytes $2 --rotate 4 --steps 30 --warmup 5 \
      --no-cpu-baseline > $O/prof_$tag.log 2>&1 || exit $?
  tail -1 $O/prof_$tag.log | cut -c1-160
done
timeout -k 10 600 bash tools/sq_small.sh $O/sq || exit $?
timeout -k 10 900 bash tools/shard_forecast.sh $P/shards 8 4 > $O/shard_forecast.log 2>&1 || exit $?
tail -16 $O/shard_forecast.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
