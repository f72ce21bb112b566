#!/bin/bash
# One GPU session: pytest -m gpu, then the bench.  Each step has its own time limit; a crash or a
# timeout (rc > 1) ends the session.  Usage: tools/gpu_session.sh TAG [pytest args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
TAG=${1:-s}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" = 0 ]; then
  [ $# -gt 0 ] || set -- tests -m gpu
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest "$@" -q -rf --timeout 300 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -25 "$OUT/pytest.log"; [ $rc -le 1 ] || exit $rc
fi
if [ "${SKIP_BENCH:-0}" = 0 ]; then
  timeout -k 10 300 python bench.py ${BENCH_ARGS:---no-cpu-baseline} > "$OUT/bench.log" 2>&1
  rc=$?; echo "bench rc=$rc"; tail -c 2500 "$OUT/bench.log"; exit $rc
fi
