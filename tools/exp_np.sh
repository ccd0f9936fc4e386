set -euo pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
for m in "--no-pipeline" "--pipeline-fixup" ""; do
  timeout -k 10 200 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline $m > gpurun_out/np.log 2>&1 || { tail -5 gpurun_out/np.log; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/np.log').read().strip().splitlines()[-1]); k=d['kernel_ms']
print('$m', round(d['value']/1e9,1), {x: round(k[x]*1e3,2) for x in ('eval','select','resolve')}, {x: round(v*1e3,2) for x,v in k['resolve_phases'].items()})"
done
