#!/bin/bash
# Shard-size sweep of k_env_step on one GPU: the automatic lanes choice at the per-GPU shard of each
# strong-scaling configuration, with A/B lines for the other integrator and for the tail handoff.
# Usage: tools/lanes_sweep.sh TAG   (outputs gpurun_out/TAG/*.log; summary on stdout)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-lanes}
mkdir -p "$OUT"
line() {  # tag  env...  -- bench args
  local tag=$1; shift; local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py --no-cpu-baseline --no-open-loop --long-window 1000 "$@" \
    > "$OUT/$tag.log" 2>&1 || exit $?
  python - "$OUT/$tag.log" "$tag" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(json.dumps({"line": sys.argv[2], "envs_per_gpu": d["config"]["envs_per_gpu"], "lanes": d["config"]["lanes_per_aircraft"],
                  "window_ms": round(d["ms_per_step"], 4), "early_ms": round(d["early_regime"]["kernel_ms"], 4),
                  "long_ms": round(d["long_window"]["kernel_ms"], 4)}), flush=True)
PY
}
for N in 8192 16384 32768 65536; do line auto_$N -- --envs $N; done
line lanes1_8192 -- --envs 8192 --lanes 1
line lanes1_16384 -- --envs 16384 --lanes 1
line lanes4_32768 -- --envs 32768 --lanes 4
line nohandoff_65536 FWSIM_TAIL_QUAD=0 -- --envs 65536
line nohandoff_8192_lanes1 FWSIM_TAIL_QUAD=0 -- --envs 8192 --lanes 1
line auto_131072 -- --envs 131072
line auto_262144 -- --envs 262144
