#!/bin/bash
# Same-box A/B of the remainder reduction split into independent Horner
# chains (BMQCRC_HORNER_CHAINS 1 = base build, 2 = variant h2, 4 = variant h4;
# tools/build_variant.sh), on the small-message configs and the headline,
# alternating builds twice.  GPU box only.
#   usage: tools/r3_ab_horner.sh <prefix>
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
p=${1:-hz}
export STEPS=100 WARMUP=10
for rep in 1 2; do
    tools/ab_configs.sh "${p}_r$rep" "base h2 h4" 1M_x_256B 64k_x_64KiB 1k_x_4KiB
done
lib=blazingmq_amd/lib
cp $lib/libbmqcrc.so /tmp/hz_base.so
for v in base h2 h4; do
    if [ "$v" = base ]; then cp /tmp/hz_base.so $lib/libbmqcrc.so; else cp $lib/variant_$v.so $lib/libbmqcrc.so; fi
    for mb in 64 128; do
        timeout -k 10 120 python3 bench.py --config 1M_x_256B --msg-bytes $mb --steps 100 --warmup 10 \
            --no-cpu-baseline > gpurun_out/${p}_tiny_${v}_$mb.log 2>&1 || { cp /tmp/hz_base.so $lib/libbmqcrc.so; exit 1; }
        echo "{\"variant\": \"$v\", \"msg_bytes\": $mb, \"bench\": $(tail -1 gpurun_out/${p}_tiny_${v}_$mb.log)}" >> gpurun_out/${p}_tiny.jsonl
    done
done
cp /tmp/hz_base.so $lib/libbmqcrc.so
