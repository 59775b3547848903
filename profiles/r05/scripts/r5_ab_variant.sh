#!/bin/bash
# round 5: a variant library (V=<name>: blazingmq_amd/lib/variant_<name>.so) against
# the product build, alternated,
# on small messages read from HBM (4 rotating copies) and two BASELINE
# configs; then the parity and fuzz suites with the variant swapped in
set -o pipefail
V=${V:?variant name}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
lib=blazingmq_amd/lib
cp $lib/libbmqcrc.so /tmp/base.so
restore() { cp /tmp/base.so $lib/libbmqcrc.so; }
out=gpurun_out/r5/${V}_ab.jsonl
: > $out
for v in base $V base $V; do
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
        2> gpurun_out/r5/${V}_${v}_$tag.err | tail -1) || rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then restore; echo "bench rc $rc"; exit $rc; fi
    echo "{\"variant\": \"$v\", \"args\": \"$args\", \"bench\": $line}" >> $out
    echo "$v $tag: $(echo "$line" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_avg_us"], d["roofline"]["frac_per_step"], d["parity"])')"
  done
done
cp $lib/variant_$V.so $lib/libbmqcrc.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q \
    --timeout 240 --timeout-method thread > gpurun_out/r5/${V}_parity.log 2>&1
rc=$?
restore
tail -3 gpurun_out/r5/${V}_parity.log
exit $rc
