mkdir -p gpurun_out
for t in 0 4 0 4; do
  for c in 1M_x_256B zipf_4M; do
    BMQCRC_TUNE=$t timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab_${c}_t${t}.log 2>&1 || exit 1
    echo "t=$t $c $(tail -1 gpurun_out/ab_${c}_t${t}.log | cut -c1-10)"
  done
done
