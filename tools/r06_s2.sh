#!/bin/bash
# Round-6 GPU session 2: the new env-draw tape tests first, then the whole GPU suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
TAG=${1:-r06s2}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_r06.py -x -v --timeout 120 --timeout-method thread > "$OUT/r06.log" 2>&1
rc=$?; tail -25 "$OUT/r06.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; exit $rc
