#!/bin/bash
# Instruction-mix PMC passes on k_env_step (65536 aircraft, fp32), one rocprofv3 run per pass.
# Normalise per RK iteration with the sweep's nfev_wave_max_mean (printed in p0.log).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=${PMC_OUT:-gpurun_out/pmc2}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=${PMC_ARGS:-"tools/sweep.py --sizes 65536 --steps 3"}
timeout -k 10 240 python $ARGS > "$OUT/p0.log" 2>&1 || exit $?
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS" \
           "SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_CVT" \
           "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP64 SQ_IFETCH SQC_ICACHE_MISSES SQC_DCACHE_MISSES"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $set --output-format csv -d "$OUT/p$i" -- python $ARGS > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -le 1 ] || exit $rc
done
python tools/pmc_report.py "$OUT"
grep nfev "$OUT/p0.log" | tail -2
