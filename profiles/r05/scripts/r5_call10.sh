#!/bin/bash
# round 5, GPU call 10: the remainder step over 5-bit conflict-free tables
# (variant_h5.so, TUNE bit 13) against the byte tables (product), alternated,
# on small messages read from HBM (4 rotating copies) and two BASELINE
# configs; then the parity and fuzz suites with the variant swapped in
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
lib=blazingmq_amd/lib
cp $lib/libbmqcrc.so /tmp/base.so
restore() { cp /tmp/base.so $lib/libbmqcrc.so; }
out=gpurun_out/r5/h5_ab.jsonl
: > $out
for v in base h5 base h5; do
  if [ $v = base ]; then restore; else cp $lib/variant_$v.so $lib/libbmqcrc.so; fi
  for w in "1048576 256 4" "4194304 256 4" "2097152 128 4" "4194304 64 4" "1048576 200 4" "zipf_4M" "64k_x_64KiB"; do
    set -- $w
    rc=0
    if [ $# -eq 3 ]; then
      args="--config 1M_x_256B --msgs $1 --msg-bytes $2 --rotate $3"; tag=$1_$2
    else
      args="--config $1"; tag=$1
    fi
    line=$(timeout -k 10 180 python bench.py $args --steps 30 --warmup 5 --no-cpu-baseline \
        2> gpurun_out/r5/h5_${v}_$tag.err | tail -1) || rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then restore; echo "bench rc $rc"; exit $rc; fi
    echo "{\"variant\": \"$v\", \"args\": \"$args\", \"bench\": $line}" >> $out
    echo "$v $tag: $(echo "$line" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_avg_us"], d["roofline"]["frac_per_step"], d["parity"])')"
  done
done
cp $lib/variant_h5.so $lib/libbmqcrc.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q \
    --timeout 240 --timeout-method thread > gpurun_out/r5/h5_parity.log 2>&1
rc=$?
restore
tail -3 gpurun_out/r5/h5_parity.log
exit $rc
