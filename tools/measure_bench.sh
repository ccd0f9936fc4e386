#!/bin/bash
# The round's headline measurement on one box: the driver's bench command three times (submit-ahead), once with one
# call per step (--sync), and once under rocprofv3 --kernel-trace --stats (tools/gpu_prof.sh).
# usage (GPU box): tools/measure_bench.sh TAG   -> gpurun_out/TAG/, gpurun_out/TAGprof/
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-measure}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > "$O/bench_driver.json" 2> "$O/bench_driver.err" || exit 1
for i in 2 3; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --stream-nodes 0 > "$O/bench_driver_rep$i.json" 2> "$O/rep$i.err" || exit 1
done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --sync --no-cpu-baseline --stream-nodes 0 > "$O/bench_driver_sync.json" 2> "$O/sync.err" || exit 1
STEPS=20 bash tools/gpu_prof.sh "${TAG}prof" > "$O/prof.txt" 2>&1 || exit 1
echo done
