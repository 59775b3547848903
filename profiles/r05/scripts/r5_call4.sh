#!/bin/bash
# round 5, GPU call 4: batches planned without a shape prediction (bench.py's
# planned leg, BMQCRC_F_PLAN) by k_plan_map (base) or by the light k_plan
# (variant_light.so, TUNE bit 12), three configs, alternated; then the
# strong-scaling shard forecast
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
lib=blazingmq_amd/lib
cp $lib/libbmqcrc.so /tmp/base.so
out=gpurun_out/r5/light_ab.jsonl
: > $out
for v in base light base light; do
  if [ $v = base ]; then cp /tmp/base.so $lib/libbmqcrc.so; else cp $lib/variant_$v.so $lib/libbmqcrc.so; fi
  for c in zipf_4M 1M_x_256B 1k_x_4KiB; do
    steps=20; [ $c = 1k_x_4KiB ] && steps=200
    rc=0
    line=$(timeout -k 10 240 python bench.py --config $c --steps $steps --warmup 5 --no-cpu-baseline \
        2> gpurun_out/r5/light_${v}_$c.err | tail -1) || rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then cp /tmp/base.so $lib/libbmqcrc.so; echo "bench rc $rc"; exit $rc; fi
    echo "{\"variant\": \"$v\", \"bench\": $line}" >> $out
    echo "$v $c: $(echo "$line" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d["planned_ms_per_step"], d["planned_kernels_per_step"], d["parity"])')"
  done
done
cp /tmp/base.so $lib/libbmqcrc.so
timeout -k 10 900 bash tools/shard_forecast.sh r5_sf 8 4 > gpurun_out/r5/shard_forecast.log 2>&1
