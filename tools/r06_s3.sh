#!/bin/bash
# Round-6 session 3: the GPU suite on the build with y / f in registers (FW_YF_REGS=1), then A/B bench lines at
# 65536 aircraft: the in-tree build, variants (tools/_build/ab), the tail-handoff threshold (FWSIM_TAIL_QUAD).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-r06s3}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
line() {  # tag  env...  -- bench args
  local tag=$1; shift; local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py --no-cpu-baseline --no-open-loop --no-fp64 --no-replay \
    --rollout-steps 0 --sac-fill-steps 0 --long-window 2000 "$@" > "$OUT/$tag.log" 2>&1 || exit $?
  python - "$OUT/$tag.log" "$tag" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(json.dumps({"line": sys.argv[2], "envs_per_gpu": d["config"]["envs_per_gpu"], "lanes": d["config"]["lanes_per_aircraft"],
                  "window_ms": round(d["ms_per_step"], 4), "early_ms": round(d["early_regime"]["kernel_ms"], 4),
                  "long_ms": round(d["long_window"]["kernel_ms"], 4)}), flush=True)
PY
}
line base -- --envs 65536
for v in yf_er yf_rhs1; do line $v FWSIM_LIB=tools/_build/ab/$v.so -- --envs 65536; done
for tq in 8 12; do line tq$tq FWSIM_TAIL_QUAD=$tq -- --envs 65536; done
line base_again -- --envs 65536
line pref_q1_check -- --envs 32768
