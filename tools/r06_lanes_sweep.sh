#!/bin/bash
# Round-6 shard-size sweep (configs[1] 4096 and configs[3]'s 8192 per GPU added): the automatic lanes choice at
# each per-GPU shard of the strong-scaling configurations, with A/B lines for the other integrators (the pair
# of round 6 included).  Usage: tools/r06_lanes_sweep.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-r06sweep}
mkdir -p "$OUT"
line() {  # tag  env...  -- bench args
  local tag=$1; shift; local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py --no-cpu-baseline --no-open-loop --no-fp64 --no-replay \
    --rollout-steps 0 --sac-fill-steps 0 --long-window 1000 "$@" > "$OUT/$tag.log" 2>&1 || exit $?
  python - "$OUT/$tag.log" "$tag" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(json.dumps({"line": sys.argv[2], "envs_per_gpu": d["config"]["envs_per_gpu"], "lanes": d["config"]["lanes_per_aircraft"],
                  "window_ms": round(d["ms_per_step"], 4), "early_ms": round(d["early_regime"]["kernel_ms"], 4),
                  "long_ms": round(d["long_window"]["kernel_ms"], 4),
                  "long_env_steps_per_s": round(d["long_window"]["env_steps_per_s"], -5)}), flush=True)
PY
}
for N in 4096 8192 16384 32768 65536; do line auto_$N -- --envs $N; done
for N in 4096 8192 16384; do line lanes1_$N -- --envs $N --lanes 1; line lanes2_$N -- --envs $N --lanes 2; done
line lanes4_32768 -- --envs 32768 --lanes 4
line lanes2_65536 -- --envs 65536 --lanes 2
# A/B: the one-lane integrator with y / f in registers instead of LDS (FW_YF_REGS=1 variant, tools/_build/ab)
for v in yfregs rhs1; do
  [ -f tools/_build/ab/$v.so ] && line ${v}_65536 FWSIM_LIB=tools/_build/ab/$v.so -- --envs 65536
done
line base_65536_again -- --envs 65536
[ -f tools/_build/ab/rhs1.so ] && line rhs1_65536_again FWSIM_LIB=tools/_build/ab/rhs1.so -- --envs 65536
