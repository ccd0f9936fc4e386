#!/bin/bash
# Round-3 measurement pass on one GPU box: the workload tools (C5 DeviceShare + quota, C4 cpusets, 8-zone NUMA)
# and a node-count sweep of bench.py (eval+select vs replay per batch, for the multi-GPU crossover).  Every GPU
# step has its own time limit and the chain stops at the first failure.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-sweep}
STEPS=${STEPS:-ds,c4,numa,nodes}
if [[ $STEPS == *ds* ]]; then
  timeout -k 10 300 python -u tools/ds_bench.py > gpurun_out/ds_$TAG.log 2>&1 || { tail -30 gpurun_out/ds_$TAG.log; exit 1; }
  tail -1 gpurun_out/ds_$TAG.log
fi
if [[ $STEPS == *c4* ]]; then
  timeout -k 10 300 python -u tools/cpuset_bench.py --survey > gpurun_out/c4_$TAG.log 2>&1 || { tail -30 gpurun_out/c4_$TAG.log; exit 1; }
  tail -1 gpurun_out/c4_$TAG.log
fi
if [[ $STEPS == *numa* ]]; then
  timeout -k 10 300 python -u tools/numa_bench.py --pods 4096 > gpurun_out/numa_$TAG.log 2>&1 || { tail -30 gpurun_out/numa_$TAG.log; exit 1; }
  tail -1 gpurun_out/numa_$TAG.log
fi
if [[ $STEPS == *nodes* ]]; then
  for n in 50000 200000 1000000; do
    timeout -k 10 300 python -u bench.py --nodes $n --pods 12800 --steps 3 --no-cpu-baseline --stream-nodes 0 \
      > gpurun_out/nodes_${n}_$TAG.log 2>&1 || { tail -30 gpurun_out/nodes_${n}_$TAG.log; exit 1; }
    tail -1 gpurun_out/nodes_${n}_$TAG.log
  done
fi
