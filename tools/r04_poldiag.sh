#!/bin/bash
# Policy-launch timing diagnostics (wrong results, timing only): shipped kernel vs no tanh (FW_POL_DIAG=1) vs no
# hidden-layer MFMA (FW_POL_DIAG=2), tools/pol_bench.py per library variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-poldiag}
mkdir -p "$OUT"
for v in ${POLDIAG:-default diag1 diag2}; do
  L=; [ "$v" != default ] && L=tools/_build/variants/$v.so
  FWSIM_LIB=$L timeout -k 10 120 python3 tools/pol_bench.py > "$OUT/$v.log" 2>&1 || exit $?
  echo "$v $(grep kernel "$OUT/$v.log" | tail -2 | tr '\n' ' ')"
done
