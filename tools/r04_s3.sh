#!/bin/bash
# Round-4 check: GPU suite, policy launch time, lone-wave tail fit, driver-window bench with the configs[2]
# collect leg.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-s3}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
  || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 120 python3 tools/pol_bench.py > "$OUT/pol.log" 2>&1 || exit $?
tail -2 "$OUT/pol.log"
timeout -k 10 200 python3 tools/tail.py > "$OUT/tail.log" 2>&1 || exit $?
tail -4 "$OUT/tail.log"
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --rollout-steps 2048 --no-fp64 --no-replay \
  > "$OUT/bench.log" 2>&1 || exit $?
tail -1 "$OUT/bench.log" | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('value', d['value'], 'ms', d['ms_per_step'], 'long', d['long_window'], 'collect', d['rollout']['env_steps_per_s'], 'open', d.get('open_loop_rollout',{}).get('value'))"
