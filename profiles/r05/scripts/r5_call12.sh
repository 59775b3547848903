#!/bin/bash
# round 5, GPU call 12: where the 1/8 Zipf shard's fixed costs go -- kernel
# trace of the shard and of the whole batch (k_plan_map and k_fold traced
# durations), and the shard at 1, 2 (auto) and 4 KiB segments
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r5/shard_costs
mkdir -p $out
for s in "--shard 0/8" "--shard 3/8" ""; do
  tag=$(echo "w$s" | tr -c 'a-z0-9\n' '_')
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_$tag -o run --output-format csv \
      -- python3 bench.py --config zipf_4M --no-cpu-baseline --steps 20 --warmup 5 $s \
      > $out/prof_$tag.log 2>&1 || exit $?
  tail -1 $out/prof_$tag.log | cut -c1-200
done
: > $out/seg_sweep.jsonl
for seg in 1024 4096 2048; do
  for s in "--shard 0/8" ""; do
    line=$(timeout -k 10 200 python3 bench.py --config zipf_4M --no-cpu-baseline --steps 20 --warmup 5 \
        --seg-bytes $seg $s 2> $out/seg.err | tail -1) || exit $?
    echo "{\"seg\": $seg, \"args\": \"$s\", \"bench\": $line}" >> $out/seg_sweep.jsonl
    echo "seg $seg $s: $(echo "$line" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d["roofline"]["kernel_avg_us"], d["parity"])')"
  done
done
