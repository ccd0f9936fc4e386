#!/bin/bash
# Round-6 measurement set on one box: the driver's bench command (submit-ahead and one call per step), the
# rocprofv3 kernel-trace stats of the bench, and the PMC passes (tools/pmc_bench.sh).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/r06"
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > "$O/bench_driver.json" 2> "$O/bench_driver.err" || exit 1
tail -c 400 "$O/bench_driver.json"; echo
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --sync --no-cpu-baseline --stream-nodes 0 > "$O/bench_driver_sync.json" 2> "$O/bench_sync.err" || exit 1
STEPS=20 bash tools/gpu_prof.sh r06prof > "$O/prof.txt" 2>&1 || exit 1
bash tools/pmc_bench.sh pmc_r06 > "$O/pmc.txt" 2>&1 || exit 1
echo done
