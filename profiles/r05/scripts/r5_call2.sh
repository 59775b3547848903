#!/bin/bash
# round 5, GPU call 2: the rolling one-segment pipeline -- its parity tests,
# then a same-box A/B against round 4's ONE loop (variant_one4.so) on
# small-message batches, every step on the next of 4 rotating copies
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 \
    --timeout-method thread -k "one_segment or speculative or declared or config_1M or golden or small_ragged" \
    > gpurun_out/r5/one_tests.log 2>&1 || exit $?
lib=blazingmq_amd/lib
cp $lib/libbmqcrc.so /tmp/base.so
out=gpurun_out/r5/one_ab.jsonl
: > $out
for v in base one4; do
  if [ $v = base ]; then cp /tmp/base.so $lib/libbmqcrc.so; else cp $lib/variant_$v.so $lib/libbmqcrc.so; fi
  for w in "1048576 256" "2097152 256" "4194304 256" "4194304 64" "2097152 128" "1048576 200"; do
    set -- $w
    rc=0
    line=$(timeout -k 10 180 python bench.py --config 1M_x_256B --msgs $1 --msg-bytes $2 --rotate 4 \
        --steps 30 --warmup 5 --no-cpu-baseline 2> gpurun_out/r5/one_ab_${v}_$1_$2.err | tail -1) || rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then cp /tmp/base.so $lib/libbmqcrc.so; echo "bench rc $rc"; exit $rc; fi
    echo "{\"variant\": \"$v\", \"msgs\": $1, \"bytes\": $2, \"bench\": $line}" >> $out
    echo "$v $1 x $2: $(echo "$line" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_avg_us"], d["roofline"]["frac"], d["roofline"]["frac_per_step"], d["parity"])')"
  done
done
cp /tmp/base.so $lib/libbmqcrc.so
