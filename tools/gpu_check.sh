#!/bin/bash
# One GPU-box pass: parity tests, bench, rocprofv3 kernel-trace summary, PMC (HBM bytes) passes on the
# eval kernel.  Every GPU step has its own time limit and the chain stops at the first failure.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-run}
STEPS=${STEPS:-tests,bench,prof,pmc}
if [[ $STEPS == *tests* ]]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests_$TAG.log 2>&1 && tail -2 gpurun_out/gpu_tests_$TAG.log || { tail -40 gpurun_out/gpu_tests_$TAG.log; exit 1; }
fi
if [[ $STEPS == *bench* ]]; then
  timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.log 2>&1 || { tail -30 gpurun_out/bench_$TAG.log; exit 1; }
  tail -1 gpurun_out/bench_$TAG.log
fi
cd /tmp && export TMPDIR=/tmp
if [[ $STEPS == *prof* ]]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$TAG" -o run -- \
    python3 "$R/bench.py" --no-cpu-baseline --stream-nodes 0 ${BENCH_ARGS:-} > "$R/gpurun_out/bench_prof_$TAG.log" 2>&1
  for f in $(find "$R/gpurun_out/prof_$TAG" -name "*kernel_stats.csv"); do cat "$f"; done
fi
if [[ $STEPS == *pmc* ]]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    for shape in "--nodes 50000 --pods 64" "--nodes 4000000 --pods 1"; do
      tag=$(echo "$c $shape" | tr -d ' -')
      mkdir -p "$R/gpurun_out/pmc_$TAG"; timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_$TAG/$tag" -o run -- \
        python3 "$R/tools/eval_probe.py" $shape --iters 10 > "$R/gpurun_out/pmc_$TAG/$tag.log" 2>&1 || { echo "pmc $tag failed"; exit 1; }
      tail -1 "$R/gpurun_out/pmc_$TAG/$tag.log"
    done
  done
fi
