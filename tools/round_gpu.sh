#!/bin/bash
# Full GPU session for a round: smoke -> gpu tests -> PMC traffic -> kernel trace -> bench.
# Each GPU step has its own time limit; the session stops at the first crash/timeout.
# Usage: tools/round_gpu.sh [tag]      (outputs under gpurun_out/<tag>/)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name timeout cmd...   (test failures rc=1 continue; crashes/timeouts stop)
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -4 "$OUT/$name.log"
  if [ $rc -gt 1 ]; then exit $rc; fi
  return 0
}
run smoke 400 python -c "import __graft_entry__ as g; g.smoke()"
run pytest_gpu 1000 python -m pytest tests -m gpu -q -rf -x
if [ "${SKIP_PROF:-0}" = 0 ]; then
  bash tools/traffic.sh > "$OUT/traffic.log" 2>&1; rc=$?; echo "traffic rc=$rc"; tail -3 "$OUT/traffic.log"; [ $rc -le 1 ] || exit $rc
  cp gpurun_out/traffic/pmc_env_step.json "$OUT/" 2>/dev/null
  run rocprof_trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -- python bench.py --no-cpu-baseline
  # the bench line's timed window = its last 1000 k_env_step dispatches
  python tools/trace_window.py "$OUT/trace" 1000 k_env_step "$OUT/trace_window.json"
fi
run bench 600 python bench.py
