#!/bin/bash
# Round-3 GPU session: gpu tests -> the driver's bench command -> its kernel trace -> nfev census.
# Each GPU step has its own time limit; a crash / timeout (rc > 1) ends the session.
# Usage: tools/r03_session.sh TAG [pytest selection...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
TAG=${1:-r03}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 "$OUT/$name.log"
  if [ $rc -gt 1 ]; then exit $rc; fi
}
if [ "${SKIP_TESTS:-0}" = 0 ]; then
  [ $# -gt 0 ] || set -- tests -m gpu
  step pytest 1100 python -u -m pytest "$@" -x -v --timeout 300 --timeout-method thread -rf
fi
if [ "${SKIP_BENCH:-0}" = 0 ]; then
  step bench_driver 400 python bench.py --gpus 1 --steps 20 --warmup 5
fi
if [ "${SKIP_TRACE:-0}" = 0 ]; then
  step trace 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
  python3 tools/driver_window.py "$OUT/trace" 20 5 1000 "$OUT/driver_window.json"
fi
if [ "${SKIP_CENSUS:-0}" = 0 ]; then
  step census 600 python tools/nfev_census.py ${CENSUS_STEPS:-4000} "$OUT/nfev_census.json"
fi
