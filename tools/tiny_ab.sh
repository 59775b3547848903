set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
lib=blazingmq_amd/lib
cp $lib/libbmqcrc.so /tmp/base.so
for rep in 1 2; do
for v in base allnt; do
  if [ $v = base ]; then cp /tmp/base.so $lib/libbmqcrc.so; else cp $lib/variant_$v.so $lib/libbmqcrc.so; fi
  for mb in 64 128 512; do
    timeout -k 10 120 python3 bench.py --config 1M_x_256B --msg-bytes $mb --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/tiny_${v}_${mb}_$rep.log 2>&1 || { cp /tmp/base.so $lib/libbmqcrc.so; exit 3; }
    echo "$v $mb $(tail -1 gpurun_out/tiny_${v}_${mb}_$rep.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["roofline"]["kernel_avg_us"], d["parity"])')"
  done
done
done
cp /tmp/base.so $lib/libbmqcrc.so
