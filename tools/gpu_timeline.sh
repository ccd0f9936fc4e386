#!/bin/bash
# Kernel timeline of a short pipelined bench run (rocprofv3 --kernel-trace, no counters), summarised per queue.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
TAG=${1:-tl}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/tl_$TAG" -o run -- \
  python3 "$R/bench.py" --no-cpu-baseline --steps 4 --warmup 1 ${BENCH_ARGS:-} > "$R/gpurun_out/tl_$TAG.log" 2>&1
f=$(find "$R/gpurun_out/tl_$TAG" -name "*kernel_trace.csv" | head -1)
python3 "$R/tools/timeline.py" "$f" | tee "$R/gpurun_out/tl_$TAG.txt"
