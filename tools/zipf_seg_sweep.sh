#!/bin/bash
# Zipf 4M whole batch and its 1/8 shard at several segment sizes (bench
# --seg-bytes; 0 = the automatic rule), one bench line each, same box.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-zss}.jsonl
: > "$out"
for seg in 0 4096 8192 16384 0; do
  for args in "" "--shard 7/8"; do
    timeout -k 10 200 python3 bench.py --config zipf_4M --no-cpu-baseline --seg-bytes $seg $args \
        > gpurun_out/zss_tmp.log 2>> gpurun_out/zss.err
    echo "{\"seg\": $seg, \"args\": \"$args\", \"bench\": $(tail -1 gpurun_out/zss_tmp.log)}" >> "$out"
    echo "seg=$seg [$args] $(tail -1 gpurun_out/zss_tmp.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d["roofline"]["kernel_avg_us"], d["parity"]["mismatches"])')"
  done
done
