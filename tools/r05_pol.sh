#!/bin/bash
# Policy kernel A/B under a kernel trace (tools/pol_bench.py, 65536 envs, SB3 default MlpPolicy, 50 launches; the
# script's own wall time per launch is host-bound, ~25 us): the in-tree library (FW_POL_TILES=1) vs
# tools/_build/variants/pt2.so (-DFW_POL_TILES=2: two 16-env tiles per wave iteration), at 2 and 3 blocks per CU
# (FW_POL_BLOCKS_PER_CU).  Prints the k_policy_mfma average duration per arm.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-r05pol}
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1 2; do
  for v in ${POL_VARIANTS:-default pt2}; do
    for b in 2 3; do
      L=; [ "$v" = default ] || L=tools/_build/variants/$v.so
      D="$OUT/${v}_b${b}_$rep"
      FWSIM_LIB=$L FW_POL_BLOCKS_PER_CU=$b timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$D" -- python3 tools/pol_bench.py > "$D.log" 2>&1 || exit $?
      f=$(find "$D" -name "*kernel_stats.csv" | head -1)
      python3 - "$f" "$v" "$b" <<'PY'
import csv, json, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "k_policy_mfma" in r["Name"]:
        print(json.dumps({"variant": sys.argv[2], "blocks_per_cu": int(sys.argv[3]), "calls": int(r["Calls"]),
                          "avg_us": round(float(r["AverageNs"]) / 1e3, 2), "min_us": round(float(r["MinNs"]) / 1e3, 2)}))
PY
    done
  done
done
