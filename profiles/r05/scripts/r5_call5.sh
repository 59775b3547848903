#!/bin/bash
# round 5, GPU call 5: where the one-segment kernel's time goes on small
# messages streamed from HBM (4 rotating copies): diagnostic builds without
# the remainder step (diag1), without the fold (diag2), without both (diag3)
# against the product, alternated; CRCs of the diagnostic builds are wrong
# by design (bench.py exits 1 on its parity check, which is expected here)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
# the planner choice changed (light k_plan without ragged evidence): the
# planner, graph, speculative and fuzz tests first
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    -k "plan or given_up or graph or shape_hint or speculative or fuzz or declared or config or share" \
    > gpurun_out/r5/planner_tests_5.log 2>&1 || exit $?
lib=blazingmq_amd/lib
cp $lib/libbmqcrc.so /tmp/base.so
out=gpurun_out/r5/one_diag.jsonl
: > $out
for v in base diag1 diag2 diag3 base diag1 diag2 diag3; do
  if [ $v = base ]; then cp /tmp/base.so $lib/libbmqcrc.so; else cp $lib/variant_$v.so $lib/libbmqcrc.so; fi
  for w in "4194304 256" "2097152 128" "4194304 64"; do
    set -- $w
    rc=0
    line=$(timeout -k 10 180 python bench.py --config 1M_x_256B --msgs $1 --msg-bytes $2 --rotate 4 \
        --steps 30 --warmup 5 --no-cpu-baseline --check 8 2> gpurun_out/r5/one_diag_${v}_$1_$2.err | tail -1) || rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then cp /tmp/base.so $lib/libbmqcrc.so; echo "bench rc $rc"; exit $rc; fi
    echo "{\"variant\": \"$v\", \"msgs\": $1, \"bytes\": $2, \"bench\": $line}" >> $out
    echo "$v $1 x $2: $(echo "$line" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_avg_us"], d["roofline"]["frac_per_step"], d["parity"])')"
  done
done
cp /tmp/base.so $lib/libbmqcrc.so
