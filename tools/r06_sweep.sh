#!/bin/bash
# Round-6 workload sweep on one box: PMC passes of the bench workload, then the reservation / DeviceShare / cpuset /
# NUMA / node-count workloads (one JSON line each under gpurun_out/r06/sweep).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/r06/sweep"
mkdir -p "$O"
cd "$R"
bash tools/pmc_bench.sh pmc_r06 > "$R/gpurun_out/r06/pmc.txt" 2>&1 || exit 1
timeout -k 10 300 python3 tools/rsv_bench.py > "$O/rsv.json" 2> "$O/rsv.err" || exit 1
timeout -k 10 300 python3 tools/ds_bench.py > "$O/ds.json" 2> "$O/ds.err" || exit 1
timeout -k 10 300 python3 tools/cpuset_bench.py > "$O/c4.json" 2> "$O/c4.err" || exit 1
timeout -k 10 300 python3 tools/numa_bench.py > "$O/numa.json" 2> "$O/numa.err" || exit 1
for n in 200000 1000000; do
  timeout -k 10 300 python3 bench.py --nodes $n --pods 12800 --steps 3 --warmup 1 --no-cpu-baseline --stream-nodes 0 > "$O/nodes_$n.json" 2> "$O/nodes_$n.err" || exit 1
done
echo done
