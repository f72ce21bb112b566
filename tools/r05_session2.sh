#!/bin/bash
# Round-5 GPU session 2: the GPU suite (all tests), then the epilogue A/B on identical states and the tail fit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
TAG=${1:-r05s2}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/epilogue_ab.py 24 > "$OUT/epilogue_ab.log" 2>&1 || exit $?
tail -1 "$OUT/epilogue_ab.log" | cut -c1-400
timeout -k 10 300 python tools/tail.py > "$OUT/tail.log" 2>&1 || exit $?
tail -1 "$OUT/tail.log" | cut -c1-500
