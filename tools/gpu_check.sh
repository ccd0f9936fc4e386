#!/bin/bash
# One GPU-box pass: parity tests, bench, rocprofv3 kernel-trace summary.  Every GPU step has its own
# time limit and the chain stops at the first failure (no retries).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-run}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/gpu_tests_$TAG.log 2>&1 && echo "tests ok" || { tail -30 gpurun_out/gpu_tests_$TAG.log; exit 1; }
timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.log 2>&1 || { tail -30 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run -- \
  python3 "$R/bench.py" --no-cpu-baseline ${BENCH_ARGS:-} > "$R/gpurun_out/bench_prof_$TAG.log" 2>&1
for f in $(find "$R/gpurun_out/prof_$TAG" -name "*kernel_stats.csv"); do cat "$f"; done
