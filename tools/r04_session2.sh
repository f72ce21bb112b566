#!/bin/bash
# Round-4 session: whole GPU suite, policy-launch A/B + counters, collect profile, traffic split, driver bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-s2}
mkdir -p "$OUT"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > "$OUT/pytest.log" 2>&1
  rc=$?; tail -1 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
fi
bash tools/r04_pol.sh "$(basename $OUT)_pol" || exit $?
SKIP_SPLIT=1 bash tools/r04_prof.sh "$(basename $OUT)_prof" || exit $?
bash tools/r04_traffic.sh "$(basename $OUT)_split" || exit $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1 || exit $?
tail -1 "$OUT/bench.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'long', d['long_window']['env_steps_per_s'], 'open', d['open_loop_rollout']['value'], 'collect', d['rollout']['env_steps_per_s'], 'fp64 long', d['fp64']['long_window'])"
