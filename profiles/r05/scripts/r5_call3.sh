#!/bin/bash
# round 5, GPU call 3: the GPU suite on the product build (incl. the
# multi-process planner test), then the no-history speculative A/B
# (variant_nohist.so, TUNE bit 11: BMQCRC_F_PLAN batches launched as the
# one-segment kernel) on the planned leg of three configs, then the
# HBM-resident (rotating) configs[1] under rocprofv3
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    > gpurun_out/r5/gpu_suite_3.log 2>&1 || exit $?
lib=blazingmq_amd/lib
cp $lib/libbmqcrc.so /tmp/base.so
out=gpurun_out/r5/nohist_ab.jsonl
: > $out
for v in base nohist base nohist; do
  if [ $v = base ]; then cp /tmp/base.so $lib/libbmqcrc.so; else cp $lib/variant_$v.so $lib/libbmqcrc.so; fi
  for c in zipf_4M 1M_x_256B 1k_x_4KiB; do
    steps=20; [ $c = 1k_x_4KiB ] && steps=200
    rc=0
    line=$(timeout -k 10 240 python bench.py --config $c --steps $steps --warmup 5 --no-cpu-baseline \
        2> gpurun_out/r5/nohist_${v}_$c.err | tail -1) || rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then cp /tmp/base.so $lib/libbmqcrc.so; echo "bench rc $rc"; exit $rc; fi
    echo "{\"variant\": \"$v\", \"bench\": $line}" >> $out
    echo "$v $c: $(echo "$line" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d["planned_ms_per_step"], d["planned_kernels_per_step"], d["parity"])')"
  done
done
cp /tmp/base.so $lib/libbmqcrc.so
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for w in "1048576 256" "2097152 256" "4194304 256" "4194304 64" "2097152 128"; do
  set -- $w
  tag=rot_$1_$2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5/prof_$tag -o run --output-format csv \
      -- python3 bench.py --config 1M_x_256B --msgs $1 --msg-bytes $2 --rotate 4 --steps 30 --warmup 5 \
      --no-cpu-baseline > gpurun_out/r5/prof_$tag.log 2>&1 || exit $?
  tail -1 gpurun_out/r5/prof_$tag.log | cut -c1-300
done
# final-build evidence: per-config bench lines, kernel traces and FETCH/WRITE
# passes (profiles/r05), the shard forecast, the smoke
timeout -k 10 1500 bash tools/profile_round.sh r5 64k_x_64KiB 1M_x_256B 16_x_256MiB zipf_4M 1k_x_4KiB \
    > gpurun_out/r5/profile_round.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5/smoke.log 2>&1
