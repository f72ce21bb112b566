#!/bin/bash
# Round-6 pair integrator session: parity tests for lanes 2, the identical-state probe (tools/pair_probe.py), then
# the bench's closed loop at 65536 and 32768 aircraft with lanes 1 and 2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
TAG=${1:-r06pair}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_r06.py tests/test_gpu_pair.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -4 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/pair_probe.py 65536 200 1000 > "$OUT/probe.json" 2> "$OUT/probe.log" || exit $?
cat "$OUT/probe.log"
for N in 65536 32768; do
  for L in 1 2; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-open-loop --no-fp64 --rollout-steps 0 --sac-fill-steps 0 \
      --no-replay --envs $N --lanes $L > "$OUT/bench_${N}_l$L.log" 2>&1 || exit $?
    python - "$OUT/bench_${N}_l$L.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(json.dumps({"envs": d["config"]["envs_per_gpu"], "lanes": d["config"]["lanes_per_aircraft"],
                  "window_ms": round(d["ms_per_step"], 4), "early_ms": round(d["early_regime"]["kernel_ms"], 4),
                  "long_ms": round(d["long_window"]["kernel_ms"], 4)}))
PY
  done
done
