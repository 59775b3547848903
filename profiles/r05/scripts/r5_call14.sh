#!/bin/bash
# round 5, GPU call 14: pipeline-depth probe for one-line groups
# (tools/depth_probe.hip) and configs[1]-shaped batches from HBM at 2M x 256 B
# on the product build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r5/call14
mkdir -p $out
timeout -k 10 240 tools/bin/depth_probe > $out/depth_probe.jsonl 2> $out/depth_probe.err || exit $?
cat $out/depth_probe.jsonl
for w in "2097152 256" "4194304 128" "1048576 256"; do
  set -- $w
  timeout -k 10 180 python bench.py --config 1M_x_256B --msgs $1 --msg-bytes $2 --rotate 4 \
      --steps 30 --warmup 5 --no-cpu-baseline > $out/rot_$1_$2.log 2>&1 || exit $?
  tail -1 $out/rot_$1_$2.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["config"]["n_msgs_total"], d["value"], d["ms_per_step"], d["roofline"]["kernel_avg_us"], d["roofline"]["frac_per_step"], d["parity"])'
done
