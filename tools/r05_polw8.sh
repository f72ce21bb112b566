#!/bin/bash
# 8-wave policy blocks (-DFW_POL_WAVES=8: four resident waves per SIMD at 128 VGPRs, one 16-env tile per wave)
# vs the in-tree 4-wave kernel: kernel-traced policy launches (tools/r05_pol.sh), then the configs[2] collect
# leg of bench.py per library, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-r05polw8}
mkdir -p "$OUT"
POL_VARIANTS="${VARS:-default w8}" bash tools/r05_pol.sh "$(basename $OUT)_pol" || exit $?
for rep in 1 2; do
  for v in ${VARS:-default w8}; do
    L=; [ "$v" = default ] || L=tools/_build/variants/$v.so
    FWSIM_LIB=$L timeout -k 10 300 python bench.py --rollout-steps 2048 --sac-fill-steps 0 --no-cpu-baseline --no-open-loop \
      --long-window 0 --no-fp64 --no-replay --steps 20 --warmup 2 --prep 100 > "$OUT/coll_$v.$rep.log" 2>&1 || exit $?
    python3 - "$OUT/coll_$v.$rep.log" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(json.dumps({"variant": sys.argv[2], "collect_env_steps_per_s": round(d["rollout"]["env_steps_per_s"] / 1e6, 1)}))
PY
  done
done
