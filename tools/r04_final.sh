#!/bin/bash
# Round-4 evidence pass: the default bench line (with the CPU baseline), the rocprofv3 kernel-trace summary and
# per-queue timeline of the same bench, and the PMC passes (one-stream schedule: counter collection serialises
# dispatches).  Every GPU step has its own time limit; the chain stops at the first failure.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-r04}
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.log 2>&1 || { tail -30 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$TAG" -o run -- \
  python3 "$R/bench.py" --no-cpu-baseline > "$R/gpurun_out/bench_prof_$TAG.log" 2>&1
f=$(find "$R/gpurun_out/prof_$TAG" -name "*kernel_trace.csv" | head -1)
python3 "$R/tools/timeline.py" "$f" > "$R/gpurun_out/timeline_$TAG.txt"
for s in $(find "$R/gpurun_out/prof_$TAG" -name "*kernel_stats.csv"); do cp "$s" "$R/gpurun_out/kernel_stats_$TAG.csv"; done
cd "$R"
bash tools/pmc_bench.sh pmc_$TAG
