#!/bin/bash
# The driver's bench command, then the configs[2] / configs[4] legs at their stated sizes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-r03legs}
mkdir -p "$OUT"
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_driver.log" 2>&1 || exit $?
tail -1 "$OUT/bench_driver.log" | cut -c1-300
timeout -k 10 600 python bench.py --rollout-steps 2048 --sac-fill-steps 1000 --no-cpu-baseline --no-fp64 --no-replay \
  --long-window 0 --no-open-loop --steps 20 --warmup 5 > "$OUT/bench_legs.log" 2>&1 || exit $?
tail -1 "$OUT/bench_legs.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({k: d.get(k) for k in ('rollout', 'sac_fill')}))"
