mkdir -p gpurun_out/cpu
for i in 1 2; do
  timeout -k 10 300 python3 bench.py > gpurun_out/cpu/bench_$i.log 2>&1 || exit 1
  tail -1 gpurun_out/cpu/bench_$i.log | python3 -c 'import json,sys; d=json.load(sys.stdin); c=d["cpu_baseline"]; print(d["value"], c["value"], c["window_spread"], c["windows_GiBps"], c["streamed_value"], c["streamed_window_spread"], c["single_thread_value"])'
done
timeout -k 10 300 python3 bench.py --config 1M_x_256B > gpurun_out/cpu/bench_256.log 2>&1 || exit 1
tail -1 gpurun_out/cpu/bench_256.log | python3 -c 'import json,sys; d=json.load(sys.stdin); c=d["cpu_baseline"]; print(d["value"], c["value"], c["window_spread"], c["windows_GiBps"], c["streamed_value"], c["streamed_window_spread"])'
