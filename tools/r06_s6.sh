#!/bin/bash
# Round-6 session 6: the attitude_angular targets (ABI 12) -- the round-6 GPU tests (reference episodes through the
# env-draw tape, incl. the new "attang" case) first, then the whole suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-r06s6}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_r06.py -x -q --timeout 300 --timeout-method thread -rf > "$OUT/r06.log" 2>&1
rc=$?; tail -15 "$OUT/r06.log" | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; exit $rc
