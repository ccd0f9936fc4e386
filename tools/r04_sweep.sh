#!/bin/bash
# Round-4 measurement pass of the other workloads: C5 DeviceShare + quota, C4 cpusets, 8-zone NUMA, the
# reservation mix (tools/rsv_bench.py) and the node-count sweep of bench.py.  Every GPU step has its own time
# limit; the chain stops at the first failure.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-r04}
STEPS=ds,c4,numa,nodes bash tools/r03_sweep.sh $TAG
timeout -k 10 300 python -u tools/rsv_bench.py > gpurun_out/rsv_$TAG.log 2>&1 || { tail -30 gpurun_out/rsv_$TAG.log; exit 1; }
tail -1 gpurun_out/rsv_$TAG.log
