#!/bin/bash
# merge kernels after a change: standalone launch times, the VecNormalize / collect GPU tests, configs[2] collect.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-mergecf}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/merge_bench.py > "$OUT/mb.log" 2>&1 || exit $?
grep '{' "$OUT/mb.log" | tail -1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "policy or collect or rollout or vecnorm or merge or moments or shard" \
  --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
timeout -k 10 400 python3 bench.py --rollout-steps 2048 --no-cpu-baseline --no-open-loop --long-window 0 \
  --no-fp64 --no-replay --steps 5 --warmup 2 --prep 100 > "$OUT/collect2048.log" 2>&1 || exit $?
tail -1 "$OUT/collect2048.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('collect2048', d['rollout']['env_steps_per_s'])"
