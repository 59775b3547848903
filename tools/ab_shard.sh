#!/bin/bash
# Same-box A/B of two library builds on Zipf: the full batch and one shard of
# an N-way strong-scaling split.  usage: tools/ab_shard.sh <prefix> <variant> [shards]
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
prefix=$1; name=$2; shards=${3:-"0/8"}
lib=blazingmq_amd/lib
cp $lib/libbmqcrc.so /tmp/ab_base.so
out=gpurun_out/$prefix.jsonl
: > $out
run() {  # tag, extra args
    rc=0
    timeout -k 10 200 python3 bench.py --config zipf_4M --no-cpu-baseline "${@:2}" \
        > gpurun_out/${prefix}_tmp.log 2>> gpurun_out/$prefix.err || rc=$?
    [ "$rc" -eq 0 ] || { echo "bench exited $rc"; exit "$rc"; }
    line=$(tail -1 gpurun_out/${prefix}_tmp.log)
    echo "{\"lib\": \"$1\", \"args\": \"${*:2}\", \"bench\": $line}" >> $out
    echo "$1 ${*:2} $(echo "$line" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_avg_us"], d["parity"]["mismatches"])')"
}
for rep in 1 2; do
    for v in A B; do
        if [ $v = A ]; then cp /tmp/ab_base.so $lib/libbmqcrc.so; else cp $lib/variant_$name.so $lib/libbmqcrc.so; fi
        run $v
        for sh in $shards; do run $v --shard $sh; done
    done
done
cp /tmp/ab_base.so $lib/libbmqcrc.so
