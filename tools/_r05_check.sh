#!/bin/bash
# round-5 working check: GPU parity of the pipelined schedule and the submit/wait API, then the bench line
# (submit-ahead and one call per step) and the eval kernel alone
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/${1:-chk}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_async.py tests/test_gpu_parity.py tests/test_gpu_ext.py > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --sync > $O/bench_sync.json 2> $O/bench_sync.err || exit 1
timeout -k 10 120 python3 tools/eval_probe.py --pods 64 --iters 50 >> $O/eval.log 2>&1 || exit 1
echo done
