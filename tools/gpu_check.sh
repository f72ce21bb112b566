#!/bin/bash
# One GPU session: smoke -> gpu tests -> short bench.  Stops at the first
# crash / timeout (exit status > 1); plain test failures (1) continue.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -5 "gpurun_out/$name.log"
  if [ $rc -gt 1 ]; then exit $rc; fi
  return 0
}
run smoke 400 python -c "import __graft_entry__ as g; g.smoke()"
run pytest_gpu 900 python -m pytest tests -m gpu -q -rf
run bench 400 python bench.py --steps 200 --warmup 20
