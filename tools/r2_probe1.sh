set -o pipefail
mkdir -p gpurun_out
for args in "256 1048576 0 0" "256 1048576 2 100" "256 1048576 3 250" "256 1048576 6 500" "256 4194304 3 250"; do
  timeout -k 5 60 tools/bin_direct_probe $args >> gpurun_out/r2_direct_probe.jsonl || exit 1
done
cat gpurun_out/r2_direct_probe.jsonl
