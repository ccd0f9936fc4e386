set -e
for args in "--zones 8 --pod-policy 0 --status 0" "--zones 8 --pod-policy 0.2 --status 0.1" "--zones 4 --pod-policy 0 --status 0" "--zones 2 --pod-policy 0 --status 0"; do
  timeout -k 10 200 python -u tools/numa_bench.py --nodes 50000 --pods 1280 --steps 2 --no-cpu-baseline $args >> gpurun_out/numa_var.log 2>&1
  tail -1 gpurun_out/numa_var.log
done
