#!/bin/bash
# round 5, GPU call 13: k_plan_map's duration on the 1/8 Zipf shard and the
# whole batch with parts of phase 2 skipped (BMQCRC_PLAN_SKIP diagnostic
# builds: 2 no last-segment claims, 4 no full-run writes, 8 no last-segment
# stores; the map is wrong there, k_fold's CRCs are not used)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r5/plan_skip
mkdir -p $out
lib=blazingmq_amd/lib
cp $lib/libbmqcrc.so /tmp/base.so
restore() { cp /tmp/base.so $lib/libbmqcrc.so; }
for v in base pskip2 pskip4 pskip8 base; do
  if [ $v = base ]; then restore; else cp $lib/variant_$v.so $lib/libbmqcrc.so; fi
  for s in "--shard 0/8" ""; do
    tag=${v}_$(echo "w$s" | tr -c 'a-z0-9\n' '_')
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/$tag -o run --output-format csv \
        -- python3 bench.py --config zipf_4M --no-cpu-baseline --steps 10 --warmup 3 $s \
        > $out/$tag.log 2>&1 || { restore; exit 1; }
    grep -h "k_plan_map" $out/$tag/run_kernel_stats.csv | cut -d, -f1-8
  done
done
restore
