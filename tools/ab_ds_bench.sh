#!/bin/bash
# Same-box A/B of evaluator builds (tools/ab_build.sh) on the config-5 DeviceShare + quota workload
# (tools/ds_bench.py), in the order given.
# usage (on the GPU box): LIBS="lib_a lib_b lib_a lib_b" bash tools/ab_ds_bench.sh
set -uo pipefail
mkdir -p gpurun_out
for L in ${LIBS}; do
  KOORDEVAL_LIB=$PWD/koordinator_amd/$L.so timeout -k 10 200 python3 tools/ds_bench.py --no-cpu-baseline > gpurun_out/dsab_$L.json 2> gpurun_out/dsab_$L.err || { tail -5 gpurun_out/dsab_$L.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/dsab_$L.json').read().strip().splitlines()[-1]); print('$L', round(d['value']/1e6,1), 'M/s resolve_ms', round(d['kernel_ms_per_batch']['resolve_ms'],3), 'eval', round(d['kernel_ms_per_batch']['eval_ms'],3))"
done
