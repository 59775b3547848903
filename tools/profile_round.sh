#!/bin/bash
# Collect the rocprofv3 evidence for every bench config on the GPU box:
#   <prefix>_<cfg>   --kernel-trace --stats      (per-kernel average duration,
#                    with bench.py's default settle phase so it matches the
#                    live HIP-event figure on a warm GPU)
#   <prefix>f_<cfg>  --pmc FETCH_SIZE             (own pass, no trace domains)
#   <prefix>w_<cfg>  --pmc WRITE_SIZE
#   bench_<cfg>.log  plain bench.py line (value, roofline, cpu_baseline)
# then summarize with tools/summarize_profiles.py in the build container.
#
# usage (on the box): tools/profile_round.sh <prefix> [config ...]
set -eo pipefail
cd /tmp && export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
prefix=$1
shift
configs=${*:-"64k_x_64KiB 1M_x_256B 16_x_256MiB zipf_4M"}
out=gpurun_out
mkdir -p $out
for c in $configs; do
    echo "== $c $(date +%T)"
    # a 1k x 4 KiB step is ~8 us: 400 steps keep the final synchronize out of it
    steps=20
    [ "$c" = 1k_x_4KiB ] && steps=400
    timeout -k 10 300 python3 bench.py --config $c --steps $steps --warmup 5 \
        > $out/bench_${prefix}_$c.log 2>&1
    tail -1 $out/bench_${prefix}_$c.log
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/${prefix}_$c -o run \
        --output-format csv -- python3 bench.py --config $c --steps 20 --warmup 5 \
        --no-cpu-baseline > $out/${prefix}_$c.log 2>&1
    timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $out/${prefix}f_$c -o run \
        --output-format csv -- python3 bench.py --config $c --steps 5 --warmup 2 \
        --no-cpu-baseline --settle-seconds 0 --no-kernel-timing > $out/${prefix}f_$c.log 2>&1
    timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $out/${prefix}w_$c -o run \
        --output-format csv -- python3 bench.py --config $c --steps 5 --warmup 2 \
        --no-cpu-baseline --settle-seconds 0 --no-kernel-timing > $out/${prefix}w_$c.log 2>&1
done
echo "== done $(date +%T)"
