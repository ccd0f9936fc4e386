#!/bin/bash
# A/B of the T-row helper workgroups (KOORDEVAL_T_HELPERS) and the patched early eval (KOORDEVAL_EVAL_PATCH):
# the GPU parity tests (defaults), then the bench per VARIANTS ("helpers:patch" pairs).  TESTS=0 skips the tests.
set -euo pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
if [[ ${TESTS:-1} == 1 ]]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/h_tests.log 2>&1 || { tail -30 gpurun_out/h_tests.log; exit 1; }
  tail -1 gpurun_out/h_tests.log
fi
for v in ${VARIANTS:-4:1 4:0 0:1}; do
  h=${v%%:*}; pt=${v##*:}
  KOORDEVAL_T_HELPERS=$h KOORDEVAL_EVAL_PATCH=$pt timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/h$h.$pt.log 2>&1 || { tail -5 gpurun_out/h$h.$pt.log; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/h$h.$pt.log').read().strip().splitlines()[-1]); k=d['kernel_ms']
print('helpers:patch $v', round(d['value']/1e9,2), {x: round(k[x]*1e3,2) for x in ('eval','select','handoff','resolve')}, {x: round(v*1e3,2) if 'hit' not in x else round(v,3) for x,v in k['resolve_phases'].items()})"
done
