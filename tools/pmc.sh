#!/bin/bash
# PMC passes on k_env_step (65536 aircraft, fp32).  Each pass is its own rocprofv3 run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
ARGS=${PMC_ARGS:-"tools/sweep.py --sizes 65536 --steps 3"}
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_DCACHE_HITS SQC_DCACHE_MISSES SQ_IFETCH SQ_INSTS_SMEM SQ_INST_CYCLES_SALU SQ_THREAD_CYCLES_VALU" \
           "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_BRANCH" \
           ${PMC_EXTRA}; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc/p$i -- python $ARGS > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -le 1 ] || exit $rc
done
python tools/pmc_report.py gpurun_out/pmc
