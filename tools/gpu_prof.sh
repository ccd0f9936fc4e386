#!/bin/bash
# Kernel-trace profile of the default bench workload: rocprofv3 stats + trace, then the timeline summary.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-prof}
mkdir -p "$R/gpurun_out/$TAG"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/$TAG" -o run -- \
  python3 "$R/bench.py" --no-cpu-baseline --stream-nodes 0 --steps ${STEPS:-10} --warmup 1 ${BENCH_ARGS:-} > "$R/gpurun_out/$TAG/bench.log" 2>&1
tail -1 "$R/gpurun_out/$TAG/bench.log"
f=$(find "$R/gpurun_out/$TAG" -name "*kernel_trace.csv" | head -1)
python3 "$R/tools/timeline.py" "$f" > "$R/gpurun_out/$TAG/timeline.txt"
s=$(find "$R/gpurun_out/$TAG" -name "*kernel_stats.csv" | head -1)
cut -d, -f1-4 "$s" | head -12
cat "$R/gpurun_out/$TAG/timeline.txt"
gzip -f "$f"
