#!/bin/bash
# Tail fit A/B of the round-5 quad-front cuts (one-reciprocal stall blend, select-free reciprocals): the in-tree
# library vs tools/_build/variants/r4front.so (-DFW_QUAD_SIGMA_1RCP=0 -DFW_QUAD_RC_NOSEL=0), alternating, on the
# round-4 protocol (400 launches after 20 warm-up steps) and on a steady-state one (1000 untimed steps first).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-tailab}
mkdir -p "$OUT"
for rep in 1 2; do
  TAIL_STEPS=400 timeout -k 10 600 python tools/ab.py run default r4front >> "$OUT/tail_ab_400.log" 2>&1 || exit $?
  TAIL_PREP=1000 TAIL_STEPS=400 timeout -k 10 600 python tools/ab.py run default r4front >> "$OUT/tail_ab_steady.log" 2>&1 || exit $?
done
cat "$OUT"/tail_ab_*.log
