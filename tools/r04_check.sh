#!/bin/bash
# Round-4 GPU session: [issue probe], the round's new tests first, then smoke, the whole GPU suite and the
# driver's bench command.  Every GPU step under its own time limit; stops at the first failure.
# Usage: tools/r04_check.sh OUTDIR [quick]   (quick: new tests + smoke + bench only)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-r04}
mkdir -p "$OUT"
if [ -x tools/_build/issue_probe ]; then
  timeout -k 10 60 tools/_build/issue_probe > "$OUT/issue_probe.log" 2>&1 || exit $?
fi
timeout -k 10 400 python -u -m pytest tests/test_gpu_r04.py -x -v --timeout 200 --timeout-method thread > "$OUT/r04.log" 2>&1
rc=$?; tail -1 "$OUT/r04.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
tail -1 "$OUT/smoke.log"
if [ "$2" != "quick" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > "$OUT/pytest.log" 2>&1
  rc=$?; tail -1 "$OUT/pytest.log"; [ $rc -le 1 ] || exit $rc
fi
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1 || exit $?
tail -1 "$OUT/bench.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'long', d['long_window']['env_steps_per_s'], 'open', d['open_loop_rollout']['value'], 'collect', d['rollout']['env_steps_per_s'])"
