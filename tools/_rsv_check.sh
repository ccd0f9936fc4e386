#!/bin/bash
# reservation-path working check: GPU parity of the reservation / lifecycle / DS tests, then the matched-path costs
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/${1:-rsv}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_reservations.py tests/test_gpu_reservation_holdings.py tests/test_gpu_lifecycle.py tests/test_gpu_parity.py tests/test_gpu_cpuset.py tests/test_gpu_ds_hints.py > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python3 tools/rsv_phases.py --reps 40 > $O/phases.json 2> $O/phases.err || exit 1
timeout -k 10 300 python3 tools/rsv_bench.py > $O/rsv.json 2> $O/rsv.err || exit 1
echo done
