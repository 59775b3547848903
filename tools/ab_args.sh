#!/bin/bash
# Same-box A/B of library builds over arbitrary bench.py argument sets (on the
# GPU box).  Every variant runs every argument set, variants alternated, the
# whole sweep repeated REPS times; one JSON line per run.
#   usage: [REPS=2] tools/ab_args.sh <prefix> "<variants>" "<tag>:<bench args>" ...
#     variant "base" = the product build, others blazingmq_amd/lib/variant_<v>.so
#     e.g. tools/ab_args.sh t1 "base r2" "256:--config 1M_x_256B" \
#          "64:--config 1M_x_256B --msg-bytes 64"
#   output: gpurun_out/<prefix>.jsonl  {"variant", "tag", "rep", "bench": <line>}
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
prefix=$1
variants=$2
shift 2
mkdir -p gpurun_out "$(dirname gpurun_out/$prefix)"
out=gpurun_out/$prefix.jsonl
: > "$out"
lib=blazingmq_amd/lib
cp $lib/libbmqcrc.so /tmp/ab_args_base.so
restore() { cp /tmp/ab_args_base.so $lib/libbmqcrc.so; }
for rep in $(seq 1 ${REPS:-2}); do
  for v in $variants; do
    if [ "$v" = base ]; then restore; else cp $lib/variant_$v.so $lib/libbmqcrc.so; fi
    for spec in "$@"; do
      tag=${spec%%:*}
      args=${spec#*:}
      log=gpurun_out/${prefix}_${v}_${tag}_$rep.log
      rc=0
      timeout -k 10 240 python3 bench.py $args --steps ${STEPS:-20} --warmup ${WARMUP:-5} \
          --no-cpu-baseline > "$log" 2>&1 || rc=$?
      # 1 = parity mismatches (diagnostic builds); anything else ends the call
      if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then
        restore
        echo "bench exited $rc ($v $tag); stopping"
        tail -5 "$log"
        exit "$rc"
      fi
      line=$(grep '^{' "$log" | tail -1)
      echo "{\"variant\": \"$v\", \"tag\": \"$tag\", \"rep\": $rep, \"bench\": $line}" >> "$out"
      echo "$line" | python3 -c 'import json,sys; d=json.load(sys.stdin); r=d["roofline"]; print("%-8s %-6s %9.1f GiB/s  k_fold %8.2f us  frac %.4f  planned %s  bad %s" % (sys.argv[1], sys.argv[2], d["value"], r["kernel_avg_us"], r["frac"], d.get("planned_ms_per_step"), d["parity"]["mismatches"]))' "$v" "$tag"
    done
  done
done
restore
