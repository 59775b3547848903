#!/bin/bash
# Bench lines for every GPU config under several library builds, one short
# bench.py run each, on the GPU box.  A variant is "base" (the product
# build) or a name built by tools/build_variant.sh (variant_<name>.so, e.g.
# with -DBMQCRC_TUNE_BITS=...); it is swapped in as libbmqcrc.so for its runs.
#   usage: [STEPS=K WARMUP=W] tools/ab_configs.sh <prefix> "<variants>" [config ...]
#   output: gpurun_out/<prefix>.jsonl, one line per (variant, config)
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
prefix=$1
variants=${2:-"base"}
shift 2 || true
configs=${*:-"64k_x_64KiB 1M_x_256B 16_x_256MiB zipf_4M"}
mkdir -p gpurun_out
out=gpurun_out/$prefix.jsonl
: > "$out"
lib=blazingmq_amd/lib
[ -f /tmp/ab_cfg_base.so ] || cp $lib/libbmqcrc.so /tmp/ab_cfg_base.so
for v in $variants; do
    if [ "$v" = base ]; then cp /tmp/ab_cfg_base.so $lib/libbmqcrc.so; else cp $lib/variant_$v.so $lib/libbmqcrc.so; fi
    for c in $configs; do
        echo "== variant=$v $c $(date +%T)"
        rc=0
        timeout -k 10 240 python3 bench.py --config "$c" --steps ${STEPS:-20} --warmup ${WARMUP:-5} \
            --no-cpu-baseline > "gpurun_out/${prefix}_${v}_$c.log" \
            2> "gpurun_out/${prefix}_${v}_$c.err" || rc=$?
        # 1 = parity mismatches reported by bench.py (diagnostic builds); anything
        # else (fault, abort, timeout) ends the GPU work of this call
        if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then
            cp /tmp/ab_cfg_base.so $lib/libbmqcrc.so
            echo "bench exited $rc; stopping"
            exit "$rc"
        fi
        line=$(tail -1 "gpurun_out/${prefix}_${v}_$c.log")
        echo "{\"variant\": \"$v\", \"bench\": $line}" >> "$out"
        echo "$line" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["roofline"]["kernel_avg_us"], d["roofline"]["frac"], d["parity"])'
    done
done
cp /tmp/ab_cfg_base.so $lib/libbmqcrc.so
