set -euo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_res
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SMEM --kernel-trace --output-format csv -d $R/gpurun_out/pmc_res/a -o run -- python3 $R/tools/prof_schedule.py --pods 4096 > $R/gpurun_out/pmc_res/a.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d $R/gpurun_out/pmc_res/b -o run -- python3 $R/tools/prof_schedule.py --pods 4096 > $R/gpurun_out/pmc_res/b.log 2>&1 || echo "pass b failed"
