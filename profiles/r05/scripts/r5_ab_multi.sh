#!/bin/bash
# round 5: several variant libraries (VARIANTS="a b": blazingmq_amd/lib/variant_<name>.so)
# against the product build, alternated in one call, on small messages read
# from HBM (4 rotating copies), Zipf (whole and a 1/8 shard) and the
# headline; the product's parity + fuzz suites run first (PARITY=0 skips)
set -o pipefail
VARIANTS=${VARIANTS:?variant names}
TAG=${TAG:-multi}
ROUNDS=${ROUNDS:-2}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r5/$TAG
mkdir -p $out
lib=blazingmq_amd/lib
cp $lib/libbmqcrc.so /tmp/base.so
restore() { cp /tmp/base.so $lib/libbmqcrc.so; }
if [ "${PARITY:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q \
      --timeout 240 --timeout-method thread > $out/base_parity.log 2>&1 || { tail -20 $out/base_parity.log; exit 1; }
  tail -2 $out/base_parity.log
fi
res=$out/ab.jsonl
: > $res
for r in $(seq $ROUNDS); do
for v in base $VARIANTS; do
  if [ $v = base ]; then restore; else cp $lib/variant_$v.so $lib/libbmqcrc.so; fi
  for w in ${CONFIGS:-"1048576:256:4" "4194304:256:4" "2097152:128:4" "4194304:64:4" "1048576:200:4" "zipf_4M" "zipf_4M:0/8" "64k_x_64KiB"}; do
    IFS=: read -r a b c <<< "$w"
    if [ -n "$c" ] && [ "$c" = 0 ]; then
      args="--config 1M_x_256B --msgs $a --msg-bytes $b"; tag=${a}_${b}_resident
    elif [ -n "$c" ]; then
      args="--config 1M_x_256B --msgs $a --msg-bytes $b --rotate $c"; tag=${a}_$b
    elif [ -n "$b" ]; then
      args="--config $a --shard $b"; tag=${a}_shard
    else
      args="--config $a"; tag=$a
    fi
    rc=0
    line=$(timeout -k 10 240 python bench.py $args --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline \
        2> $out/${v}_$tag.err | tail -1) || rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then restore; echo "bench rc $rc ($v $tag)"; exit $rc; fi
    echo "{\"variant\": \"$v\", \"round\": $r, \"args\": \"$args\", \"bench\": $line}" >> $res
    echo "$v $tag: $(echo "$line" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_avg_us"], d["roofline"]["frac_per_step"], d["parity"]["mismatches"])')"
  done
done
done
restore
for v in ${PARITY_VARIANTS:-}; do
  cp $lib/variant_$v.so $lib/libbmqcrc.so
  timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q \
      --timeout 240 --timeout-method thread > $out/${v}_parity.log 2>&1
  rc=$?
  restore
  tail -2 $out/${v}_parity.log
  [ $rc -eq 0 ] || exit $rc
done
