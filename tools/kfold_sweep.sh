#!/bin/bash
# Traced k_fold duration vs batch size (rocprofv3 --kernel-trace --stats, one
# run per point): the slope is the per-group cost, the intercept the
# per-launch fixed cost (prologue, first memory round trips, last group).
#   usage (GPU box): tools/kfold_sweep.sh <prefix> <config> "<msg counts>" [msg bytes]
#   output: gpurun_out/<prefix>.jsonl, one line per point
set -eo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
prefix=$1; cfg=$2; counts=$3; mb=${4:-}
mkdir -p gpurun_out
: > gpurun_out/$prefix.jsonl
for n in $counts; do
    d=gpurun_out/${prefix}_$n
    timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- \
        python3 bench.py --config $cfg --msgs $n ${mb:+--msg-bytes $mb} --steps 50 --warmup 5 \
        --no-cpu-baseline --check 16 --no-kernel-timing > $d.log 2>&1
    python3 - "$d" "$n" "$cfg" "${mb:-0}" >> gpurun_out/$prefix.jsonl <<'PY'
import csv, json, sys
d, n, cfg, mb = sys.argv[1], int(sys.argv[2]), sys.argv[3], int(sys.argv[4])
rows = list(csv.DictReader(open(d + "/run_kernel_stats.csv")))
line = json.loads([x for x in open(d + ".log").read().splitlines() if x.startswith('{"metric"')][-1])
out = {"config": cfg, "msgs": n, "msg_bytes": mb or None,
       "payload_bytes": line["config"]["payload_bytes_total"],
       "ms_per_step": line["ms_per_step"],
       "kernels": {r["Name"]: {"calls": int(r["Calls"]), "avg_us": round(float(r["AverageNs"]) / 1e3, 3),
                               "min_us": round(float(r["MinNs"]) / 1e3, 3)} for r in rows}}
print(json.dumps(out))
PY
    tail -1 gpurun_out/$prefix.jsonl | cut -c1-300
done
