#!/bin/bash
# rocprofv3 PMC passes over the bench workload, one counter group per run (MI355X_MICROARCH.md "rocprofv3
# PMC slots": FETCH_SIZE and WRITE_SIZE cannot share a pass; <= 8 SQ counters per pass).  Counter collection
# serialises dispatches, so the bench runs its one-stream schedule (--no-pipeline): the persistent Reserve
# chain of the pipelined schedule waits on the eval stream and cannot run serialised.
# Usage: tools/pmc_bench.sh TAG [bench args...]; summaries: tools/pmc_summary.py gpurun_out/TAG
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-pmc}
shift || true
ARGS=${*:---pods 6400 --steps 2}
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run_pass() {
  local name=$1
  shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- \
    python3 "$R/bench.py" --no-cpu-baseline --stream-nodes 0 --warmup 0 --profile-every 0 --no-pipeline $ARGS \
    > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
run_pass fetch FETCH_SIZE &&
run_pass write WRITE_SIZE &&
run_pass sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE &&
run_pass wait SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM GRBM_GUI_ACTIVE
