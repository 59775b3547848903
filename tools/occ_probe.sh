mkdir -p gpurun_out
for t in 0 2; do
  for c in 1M_x_256B 64k_x_64KiB zipf_4M; do
    BMQCRC_TUNE=$t timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/occ_${c}_t${t}.log 2>&1 || exit 1
  done
done
