#!/bin/bash
# Round-6 session 4: A/B of y / f in registers (in-tree, FW_YF_REGS=1) against the LDS slots (noyf variant) and
# the error sum in registers too (yf_er), on the same steady-state windows (1000 and 3000 steps).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-r06s4}
mkdir -p "$OUT"
line() {
  local tag=$1; shift; local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py --no-cpu-baseline --no-open-loop --no-fp64 --no-replay \
    --rollout-steps 0 --sac-fill-steps 0 "$@" > "$OUT/$tag.log" 2>&1 || exit $?
  python - "$OUT/$tag.log" "$tag" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(json.dumps({"line": sys.argv[2], "envs_per_gpu": d["config"]["envs_per_gpu"], "window_ms": round(d["ms_per_step"], 4),
                  "early_ms": round(d["early_regime"]["kernel_ms"], 4), "long_ms": round(d["long_window"]["kernel_ms"], 4),
                  "long_steps": d["long_window"]["steps"]}), flush=True)
PY
}
for W in 1000 3000; do
  line yf_L$W -- --long-window $W
  line noyf_L$W FWSIM_LIB=tools/_build/ab/noyf.so -- --long-window $W
  line yf_er_L$W FWSIM_LIB=tools/_build/ab/yf_er.so -- --long-window $W
done
line yf_32768 -- --envs 32768
line noyf_32768 FWSIM_LIB=tools/_build/ab/noyf.so -- --envs 32768
