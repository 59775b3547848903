set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r2_segsweep2.jsonl
for mb in 8192 4096 2048; do
  for seg in 2048 4096 8192 16384; do
    timeout -k 10 200 python3 bench.py --config 64k_x_64KiB --msg-bytes $mb --seg-bytes $seg --no-cpu-baseline --check 32 > gpurun_out/r2_ss2.log 2>&1 || exit 1
    tail -1 gpurun_out/r2_ss2.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('msg', $mb, 'seg', $seg, d['ms_per_step'], d['roofline']['kernel_avg_us'], d['roofline']['frac'], d['parity'])" | tee -a gpurun_out/r2_segsweep2.jsonl
  done
done
