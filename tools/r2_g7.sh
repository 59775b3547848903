set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r2_shardseg.jsonl
for seg in 0 2048 4096 8192 32768; do
  for sh in 7/8 ""; do
    if [ -n "$sh" ]; then extra="--shard $sh"; else extra=""; fi
    timeout -k 10 200 python3 bench.py --config zipf_4M $extra --seg-bytes $seg --no-cpu-baseline --check 64 > gpurun_out/r2_ss.log 2>&1 || exit 1
    tail -1 gpurun_out/r2_ss.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('$seg', '$sh', d['ms_per_step'], d['roofline']['kernel_avg_us'], d['roofline']['frac'], d['parity'])" | tee -a gpurun_out/r2_shardseg.jsonl
  done
done
