set -euo pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
for e in 0 1 2 3; do
  if [[ $e == 0 ]]; then unset KOORDEVAL_LIB; else export KOORDEVAL_LIB=$PWD/koordinator_amd/libkoordeval_exp$e.so; fi
  timeout -k 10 200 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/exp$e.log 2>&1 || { tail -5 gpurun_out/exp$e.log; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/exp$e.log').read().strip().splitlines()[-1]); k=d['kernel_ms']['resolve_phases']
print('exp$e', round(d['value']/1e9,1), {x: round(v*1e3,2) for x,v in k.items()})"
done
