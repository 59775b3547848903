# Round-3 evidence beside the profile round: strong-scaling forecast (every
# Zipf shard, 8- and 4-way), 64/128/512-byte messages, SQ buckets of k_fold,
# the 8-rank rehearsal on one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r3x
bash tools/shard_forecast.sh ${1:-sf1} 8 4 || exit $?
for mb in 64 128 512; do
  timeout -k 10 120 python3 bench.py --config 1M_x_256B --msg-bytes $mb --steps 20 --warmup 5 \
      --no-cpu-baseline > gpurun_out/r3x/tiny_$mb.log 2>&1 || exit $?
  python3 tools/bench_summary.py gpurun_out/r3x/tiny_$mb.log
done
bash tools/sq_counters.sh ${2:-sq1} 1M_x_256B zipf_4M 64k_x_64KiB || exit $?
timeout -k 10 580 python3 tools/rehearse_ranks.py 8 gpurun_out/r3x/rehearsal_gpus8.json
