#!/bin/bash
# Long-window A/B (the bench's schedule: 1000 prep steps, 20 timed, 1000-step long window; fp32, 65536 aircraft)
# of library variants: "default" = the in-tree library, otherwise tools/_build/variants/NAME.so.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-longwin}
shift
mkdir -p "$OUT"
for rep in 1 2; do
  for v in "$@"; do
    L=; [ "$v" = default ] || L=tools/_build/variants/$v.so
    FWSIM_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --rollout-steps 0 \
      --sac-fill-steps 0 --no-fp64 --no-open-loop > "$OUT/$v.$rep.json" 2> "$OUT/$v.$rep.err" || exit $?
    python3 - "$OUT/$v.$rep.json" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
w = d["window"]["long"]["launch_ms"]
print(json.dumps({"variant": sys.argv[2], "value": round(d["value"] / 1e6, 1), "early_ms": round(d["early_regime"]["kernel_ms"], 4),
                  "long_ms": round(d["long_window"]["kernel_ms"], 4), "long_p50_ms": round(w["p50"], 4)}), flush=True)
PY
  done
done
