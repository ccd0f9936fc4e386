#!/bin/bash
# The workload sweep on one box: PMC passes of the bench workload (tools/pmc_bench.sh), then the reservation /
# DeviceShare (C5) / cpuset (C4, SURVEY.md §8d shape) / NUMA-policy / node-count workloads, one JSON line each.
# usage (GPU box): tools/sweep_workloads.sh TAG   -> gpurun_out/TAG/sweep/, gpurun_out/pmc_TAG/
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-sweep}
O="$R/gpurun_out/$TAG/sweep"
mkdir -p "$O"
cd "$R"
bash tools/pmc_bench.sh "pmc_$TAG" > "$R/gpurun_out/$TAG/pmc.txt" 2>&1 || exit 1
timeout -k 10 300 python3 tools/rsv_bench.py > "$O/rsv.json" 2> "$O/rsv.err" || exit 1
timeout -k 10 300 python3 tools/ds_bench.py > "$O/ds.json" 2> "$O/ds.err" || exit 1
timeout -k 10 300 python3 tools/cpuset_bench.py --survey > "$O/c4.json" 2> "$O/c4.err" || exit 1
timeout -k 10 300 python3 tools/numa_bench.py --pods 4096 > "$O/numa.json" 2> "$O/numa.err" || exit 1
for n in 200000 1000000; do
  timeout -k 10 300 python3 bench.py --nodes $n --pods 12800 --steps 3 --warmup 1 --no-cpu-baseline --stream-nodes 0 > "$O/nodes_$n.json" 2> "$O/nodes_$n.err" || exit 1
done
echo done
