#!/bin/bash
# k_policy_mfma duration vs batch size (kernel trace of tools/pol_bench.py at POL_N envs): fixed vs per-tile cost.
# POLN_LIBS: library variants to scan (default: the in-tree one).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-r05poln}
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in ${POLN_LIBS:-default}; do
  L=; [ "$v" = default ] || L=tools/_build/variants/$v.so
  for nn in ${POLN_SIZES:-65536 32768 16384 8192 2048 256}; do
    D="$OUT/${v}_n$nn"
    FWSIM_LIB=$L POL_N=$nn timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$D" -- python3 tools/pol_bench.py > "$D.log" 2>&1 || exit $?
    f=$(find "$D" -name "*kernel_stats.csv" | head -1)
    python3 - "$f" "$nn" "$v" <<'PY'
import csv, json, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "k_policy_mfma" in r["Name"]:
        print(json.dumps({"variant": sys.argv[3], "n": int(sys.argv[2]), "avg_us": round(float(r["AverageNs"]) / 1e3, 2),
                          "min_us": round(float(r["MinNs"]) / 1e3, 2)}))
PY
  done
done
