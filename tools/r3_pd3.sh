# k_plan_map per-block phase stamps (diagnostic builds variant_pd3.so: the
# product kernel with stamps; variant_pd4.so: the same without seginfo stores).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=blazingmq_amd/lib
cp $L/libbmqcrc.so /tmp/pd3_base.so
rc=0
for v in pd3 pd4 pd5 pd3h; do
  cp $L/variant_$v.so $L/libbmqcrc.so
  for s in 0/1 7/8; do
    echo "{\"variant\": \"$v\"}" >> gpurun_out/pd3.jsonl
    timeout -k 10 120 python3 tools/plan_trace_diag.py $s >> gpurun_out/pd3.jsonl 2> gpurun_out/pd3.err || { rc=$?; break 2; }
  done
done
cp /tmp/pd3_base.so $L/libbmqcrc.so
cat gpurun_out/pd3.jsonl
exit $rc
