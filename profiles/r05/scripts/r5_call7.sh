#!/bin/bash
# round 5, GPU call 7: load policy of one- and two-line groups on batches
# read from HBM (4 rotating copies): default policy (product) against
# non-temporal (variant_ntshort.so, TUNE bit 5), alternated
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
lib=blazingmq_amd/lib
cp $lib/libbmqcrc.so /tmp/base.so
out=gpurun_out/r5/ntshort_ab.jsonl
: > $out
for v in base ntshort base ntshort; do
  if [ $v = base ]; then cp /tmp/base.so $lib/libbmqcrc.so; else cp $lib/variant_$v.so $lib/libbmqcrc.so; fi
  for w in "1048576 256" "4194304 256" "2097152 128" "4194304 64" "1048576 200"; do
    set -- $w
    rc=0
    line=$(timeout -k 10 180 python bench.py --config 1M_x_256B --msgs $1 --msg-bytes $2 --rotate 4 \
        --steps 30 --warmup 5 --no-cpu-baseline 2> gpurun_out/r5/ntshort_${v}_$1_$2.err | tail -1) || rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then cp /tmp/base.so $lib/libbmqcrc.so; echo "bench rc $rc"; exit $rc; fi
    echo "{\"variant\": \"$v\", \"msgs\": $1, \"bytes\": $2, \"bench\": $line}" >> $out
    echo "$v $1 x $2: $(echo "$line" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_avg_us"], d["roofline"]["frac_per_step"], d["parity"])')"
  done
done
cp /tmp/base.so $lib/libbmqcrc.so
