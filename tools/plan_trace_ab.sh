#!/bin/bash
# Planner kernel times under rocprofv3 for several library builds (on the box):
# the Zipf batch and its 1/8 shard, --kernel-trace --stats only.
#   usage: tools/plan_trace_ab.sh <prefix> "<variants>"   (base = the product build)
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
prefix=$1
variants=${2:-base}
L=blazingmq_amd/lib
[ -f /tmp/pt_base.so ] || cp $L/libbmqcrc.so /tmp/pt_base.so
i=0
for v in $variants; do
    i=$((i + 1))
    if [ "$v" = base ]; then cp /tmp/pt_base.so $L/libbmqcrc.so; else cp $L/variant_$v.so $L/libbmqcrc.so; fi
    for args in "" "--shard 7/8"; do
        tag=$(echo "$i $v $args" | tr ' /' '__')
        echo "== $v $args $(date +%T)"
        timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${prefix}_$tag -o run \
            --output-format csv -- python3 bench.py --config zipf_4M --steps 20 --warmup 5 \
            --no-cpu-baseline $args > gpurun_out/${prefix}_$tag.log 2>&1
    done
done
cp /tmp/pt_base.so $L/libbmqcrc.so
