#!/bin/bash
# A/B of library builds at the per-GPU shard sizes of the strong-scaling configurations (closed loop,
# automatic lanes): window / early / long-window kernel ms per build and shard size.
# Usage: tools/ab_lanes.sh TAG LIB...   (LIB "default" = lib/libfwsim.so; GPU)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-ab_lanes}
shift
mkdir -p "$OUT"
for rep in 1 2; do
  for lib in "$@"; do
    for N in ${AB_SIZES:-8192 65536}; do
      tag=$(basename "$lib" .so)_${N}_$rep
      if [ "$lib" = default ]; then L=; else L=$lib; fi
      FWSIM_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-open-loop --no-weak --envs "$N" \
        > "$OUT/$tag.log" 2>&1 || exit $?
      python - "$OUT/$tag.log" "$tag" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(json.dumps({"line": sys.argv[2], "envs_per_gpu": d["config"]["envs_per_gpu"], "lanes": d["config"]["lanes_per_aircraft"],
                  "window_ms": round(d["ms_per_step"], 4), "early_ms": round(d["early_regime"]["kernel_ms"], 4),
                  "long_ms": round(d["long_window"]["kernel_ms"], 4)}), flush=True)
PY
    done
  done
done
