#!/bin/bash
# Round-5 review items 1 and 4, A/B on the GPU (variants built by tools/ab.py build, see profiles/README.md):
#   fold2  -DFW_QUAD_DIAG_FOLD=2: the quad's trial-step folds on 2 of 3 pairs (the fold load of an 8-lane group;
#          wrong results, timing only) -> the tail slope an 8-lane straggler group could reach through the folds
#   nho    -DFW_TAIL_QUAD=0: the shipped one-lane kernel without the tail handoff
#   hw1    + -DFW_HALF_WAVE=1: 32 aircraft per wave (2048 waves), one wave per SIMD (347 registers)
#   hw2    + -DFW_MIN_WAVES=2: the same capped at 256 registers, two resident waves per SIMD
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-r05ab2}
mkdir -p "$OUT"
export TMPDIR=/tmp
V=tools/_build/variants
for rep in 1 2; do
  TAIL_STEPS=400 timeout -k 10 600 python tools/ab.py run default fold2 >> "$OUT/fold8_400.log" 2>&1 || exit $?
done
for rep in 1 2; do
  TAIL_STEPS=200 timeout -k 10 600 python tools/ab.py run nho hw1 hw2 default >> "$OUT/halfwave_early.log" 2>&1 || exit $?
  TAIL_PREP=1000 TAIL_STEPS=200 timeout -k 10 600 python tools/ab.py run nho hw1 hw2 default >> "$OUT/halfwave_steady.log" 2>&1 || exit $?
done
for v in nho hw2; do
  FWSIM_LIB=$V/$v.so TAIL_STEPS=40 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d "$OUT/pmc_$v" -- python3 tools/tail.py > "$OUT/pmc_$v.log" 2>&1 || exit $?
done
cat "$OUT"/fold8_400.log "$OUT"/halfwave_*.log
