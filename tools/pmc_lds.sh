#!/bin/bash
# One rocprofv3 PMC pass of LDS / wait counters over the serial bench (k_select's pass-2 histogram):
# SQ_INSTS_LDS, SQ_LDS_BANK_CONFLICT (extra LDS cycles), SQ_LDS_IDX_ACTIVE (all LDS-array cycles),
# SQ_WAIT_INST_LDS, SQ_WAIT_ANY, SQ_WAVE_CYCLES, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE.
# Usage: tools/pmc_lds.sh TAG [bench args...]
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-lds}
shift || true
ARGS=${*:---pods 6400 --steps 2}
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY \
  SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$OUT/lds" -o run -- \
  python3 "$R/bench.py" --no-cpu-baseline --stream-nodes 0 --warmup 0 --profile-every 0 --no-pipeline $ARGS > "$OUT/lds.log" 2>&1
echo "lds rc=$?"
