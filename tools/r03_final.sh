#!/bin/bash
# Round-3 evidence pass at HEAD: GPU tests, the default bench line, rocprof kernel stats of the bench, replay
# phases (C3 and C5 shapes, diagnostic build), and the workload tools.  Every GPU step has its own time limit
# and the chain stops at the first failure.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-final}
STEPS=tests,bench,prof bash tools/gpu_check.sh $TAG
KOORDEVAL_LIB=koordinator_amd/libkoordeval_prof.so timeout -k 10 300 python tools/replay_phases.py > gpurun_out/phases_c3_$TAG.json
KOORDEVAL_LIB=koordinator_amd/libkoordeval_prof.so timeout -k 10 300 python tools/replay_phases.py --nodes 20000 --pods 4096 --ds 0.5 > gpurun_out/phases_c5_$TAG.json
STEPS=ds,c4,numa,nodes bash tools/r03_sweep.sh $TAG
