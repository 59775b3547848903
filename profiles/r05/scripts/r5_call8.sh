#!/bin/bash
# round 5, GPU call 8: whole-line short groups read non-temporally (product)
# against round 4's default policy for every short group (variant_r4pol.so),
# alternated, on batches read from HBM (4 rotating copies) and on the BASELINE
# configs; then the HBM-resident LDS-DMA pattern probe
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
lib=blazingmq_amd/lib
cp $lib/libbmqcrc.so /tmp/base.so
out=gpurun_out/r5/wholelines_ab.jsonl
: > $out
for v in base r4pol base r4pol; do
  if [ $v = base ]; then cp /tmp/base.so $lib/libbmqcrc.so; else cp $lib/variant_$v.so $lib/libbmqcrc.so; fi
  for w in "1048576 256 4" "4194304 256 4" "2097152 128 4" "4194304 64 4" "1048576 200 4" "zipf_4M" "64k_x_64KiB" "1M_x_256B"; do
    set -- $w
    rc=0
    if [ $# -eq 3 ]; then
      args="--config 1M_x_256B --msgs $1 --msg-bytes $2 --rotate $3"; tag=$1_$2
    else
      args="--config $1"; tag=$1
    fi
    line=$(timeout -k 10 180 python bench.py $args --steps 30 --warmup 5 --no-cpu-baseline \
        2> gpurun_out/r5/wl_${v}_$tag.err | tail -1) || rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then cp /tmp/base.so $lib/libbmqcrc.so; echo "bench rc $rc"; exit $rc; fi
    echo "{\"variant\": \"$v\", \"args\": \"$args\", \"bench\": $line}" >> $out
    echo "$v $tag: $(echo "$line" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_avg_us"], d["roofline"]["frac_per_step"], d["parity"])')"
  done
done
cp /tmp/base.so $lib/libbmqcrc.so
timeout -k 10 200 ./tools/bin_dma_hbm_probe > gpurun_out/r5/dma_hbm_probe2.jsonl 2>&1
