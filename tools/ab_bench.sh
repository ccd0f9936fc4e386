#!/bin/bash
# Same-box A/B of evaluator builds (tools/ab_build.sh): the default bench, alternating A B A B.
# usage (on the GPU box): tools/ab_bench.sh lib_a lib_b [rounds]
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
A=$1; B=$2; N=${3:-2}
for i in $(seq 1 "$N"); do
  for L in "$A" "$B"; do
    KOORDEVAL_LIB=$R/koordinator_amd/$L.so timeout -k 10 200 python3 "$R/bench.py" --steps 20 --warmup 2 --no-cpu-baseline \
      --stream-nodes 0 --profile-every 0 > "$R/gpurun_out/ab_$L.log" 2>&1 || { tail -5 "$R/gpurun_out/ab_$L.log"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$R/gpurun_out/ab_$L.log').read().strip().splitlines()[-1]); k=d['kernel_ms']; print('$L', round(d['value']/1e9,2), 'G/s replay_us', round(k['resolve_replay']*1e3,1), 'handoff_us', round(k['handoff']*1e3,1))"
  done
done
