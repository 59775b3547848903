#!/bin/bash
# A/B bench lines for every GPU config under several BMQCRC_TUNE knob values
# (see BatchArgs::tune), one short bench.py run each, on the GPU box.
#   usage: tools/ab_configs.sh <prefix> "<tune values>" [config ...]
#   output: gpurun_out/<prefix>.jsonl, one line per (tune, config)
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
prefix=$1
tunes=${2:-"0"}
shift 2 || true
configs=${*:-"64k_x_64KiB 1M_x_256B 16_x_256MiB zipf_4M"}
mkdir -p gpurun_out
out=gpurun_out/$prefix.jsonl
: > "$out"
for t in $tunes; do
    for c in $configs; do
        echo "== tune=$t $c $(date +%T)"
        rc=0
        BMQCRC_TUNE=$t timeout -k 10 240 python3 bench.py --config "$c" --steps 20 --warmup 5 \
            --no-cpu-baseline > "gpurun_out/${prefix}_${t}_$c.log" \
            2> "gpurun_out/${prefix}_${t}_$c.err" || rc=$?
        # 1 = parity mismatches reported by bench.py (diagnostic knobs); anything
        # else (fault, abort, timeout) ends the GPU work of this call
        if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then
            echo "bench exited $rc; stopping"
            exit "$rc"
        fi
        line=$(tail -1 "gpurun_out/${prefix}_${t}_$c.log")
        echo "{\"tune\": $t, \"bench\": $line}" >> "$out"
        echo "$line" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["roofline"]["kernel_avg_us"], d["roofline"]["frac"], d["parity"])'
    done
done
