#!/bin/bash
# A/B of the two pipelined schedules on one GPU box: the GPU parity tests, then bench.py with stale lists
# (default) and with k_fixup (--pipeline-fixup); prints the per-batch kernel / replay phase split of each.
# TESTS=0 skips the tests.
set -euo pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
if [[ ${TESTS:-1} == 1 ]]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
  tail -1 gpurun_out/ab_tests.log
fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_stale.log 2>&1 || { tail -20 gpurun_out/ab_stale.log; exit 1; }
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --pipeline-fixup > gpurun_out/ab_fixup.log 2>&1 || { tail -20 gpurun_out/ab_fixup.log; exit 1; }
python - <<'PY'
import json
for t in ("stale", "fixup"):
    d = json.loads(open(f"gpurun_out/ab_{t}.log").read().strip().splitlines()[-1])
    k = d["kernel_ms"]
    print(t, round(d["value"] / 1e9, 2), {x: round(k[x] * 1e3, 2) for x in ("eval", "select", "fixup", "handoff", "resolve")},
          {x: round(v * 1e3, 2) for x, v in k["resolve_phases"].items()})
PY
