#!/bin/bash
# Strong-scaling forecast on one GPU: time every shard
# of the Zipf batch's N-way byte-balanced split (what each of N ranks runs)
# and the whole batch, on the same box, one bench line each.
#   usage (on the box): tools/shard_forecast.sh <prefix> [N ...]
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
prefix=$1; shift
out=gpurun_out/$prefix.jsonl
: > "$out"
run() {
    timeout -k 10 200 python3 bench.py --config zipf_4M --no-cpu-baseline --steps 20 --warmup 5 "$@" \
        > gpurun_out/${prefix}_tmp.log 2>> gpurun_out/$prefix.err
    echo "{\"args\": \"$*\", \"bench\": $(tail -1 gpurun_out/${prefix}_tmp.log)}" >> "$out"
    tail -1 gpurun_out/${prefix}_tmp.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d["parity"])'
}
run
for n in ${*:-8 4}; do
    for ((i = 0; i < n; ++i)); do
        echo -n "shard $i/$n: "
        run --shard $i/$n
    done
done
run
