#!/bin/bash
# Policy-launch timing diagnostics (results wrong, timing only).  Build the variants first (CPU):
#   for k in 1 2 3 4; do python tools/ab.py build diag$k -DFW_POL_DIAG=$k; done
# (1 = no tanh, 2 = no hidden-layer MFMA, 3 = no LDS weight fill, 4 = no output stores; fw_rollout.hip), then
# drop ./tools/_build/variants from .gpurunignore for the run.  tools/pol_bench.py per library variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-poldiag}
mkdir -p "$OUT"
for v in ${POLDIAG:-default diag1 diag2}; do
  L=; [ "$v" != default ] && L=tools/_build/variants/$v.so
  FWSIM_LIB=$L timeout -k 10 120 python3 tools/pol_bench.py > "$OUT/$v.log" 2>&1 || exit $?
  echo "$v $(grep kernel "$OUT/$v.log" | tail -2 | tr '\n' ' ')"
done
