#!/bin/bash
# Round-5 evidence pass: the default bench line (with the CPU baseline), the rocprofv3 kernel-trace summary and
# per-queue timeline of the same bench, the PMC passes (one-stream schedule: counter collection serialises
# dispatches), then the whole -m gpu suite.  Every GPU step has its own time limit; the chain stops at the first
# failure.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-r05}
bash tools/r04_final.sh $TAG
timeout -k 10 900 python3 -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -3 gpurun_out/gpu_tests_$TAG.log
