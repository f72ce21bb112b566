#!/bin/bash
# Policy-launch A/B and counters (tools/pol_bench.py): MFMA vs VALU kernel, grid sizes, PMC on the MFMA kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-pol}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() { timeout -k 10 120 "$@" >> "$OUT/ab.log" 2>&1 || exit $?; tail -1 "$OUT/ab.log"; }
run python3 tools/pol_bench.py
FW_POL_VALU=1 run python3 tools/pol_bench.py
FW_POL_BLOCKS_PER_CU=2 run python3 tools/pol_bench.py
FW_POL_BLOCKS_PER_CU=4 run python3 tools/pol_bench.py
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY" \
           "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d "$OUT/pmc$i" -- python3 tools/pol_bench.py > "$OUT/pmc$i.log" 2>&1
  echo "pmc$i rc=$?"
done
