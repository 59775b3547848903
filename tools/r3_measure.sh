# Round-3 measurements on the box that need no kernel change:
#   1. the 8-rank bench path rehearsed on one GPU (wall time, peak host RSS)
#   2. end-to-end (staged and zero-copy) for configs[1] and configs[2]
#   3. the 8(f) protocol callers
#   4. 64 / 128 / 512-byte messages (bench.py --msg-bytes)
# Each GPU step has its own time limit; the first failure ends the call.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r3m
mkdir -p $out
steps=${*:-"rehearsal e2e protocol tiny"}
for s in $steps; do
  echo "== $s $(date +%T)"
  case $s in
  rehearsal)
    timeout -k 10 580 python3 tools/rehearse_ranks.py 8 $out/rehearsal_gpus8.json ;;
  e2e)
    for c in 1M_x_256B 64k_x_64KiB; do
      timeout -k 10 300 python3 bench.py --e2e --config $c --steps 10 --warmup 3 \
          --no-cpu-baseline > $out/e2e_$c.log 2>&1
      tail -2 $out/e2e_$c.log
    done ;;
  protocol)
    timeout -k 10 400 python3 bench.py --protocol > $out/protocol.log 2>&1
    tail -5 $out/protocol.log ;;
  tiny)
    for mb in 64 128 512; do
      timeout -k 10 120 python3 bench.py --config 1M_x_256B --msg-bytes $mb --steps 20 \
          --warmup 5 --no-cpu-baseline > $out/tiny_$mb.log 2>&1
      python3 tools/bench_summary.py $out/tiny_$mb.log
    done ;;
  esac
done
echo "== done $(date +%T)"
