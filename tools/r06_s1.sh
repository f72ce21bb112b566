#!/bin/bash
# Round-6 GPU session 1: VALU issue costs (tools/issue_probe.hip: one wave alone, one and two waves per
# SIMD), the GPU suite on the round-6 hygiene build, a short bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
TAG=${1:-r06s1}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 tools/_build/issue_probe > "$OUT/issue_probe.log" 2>&1 || exit $?
cat "$OUT/issue_probe.log"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline --rollout-steps 0 --sac-fill-steps 0 --no-fp64 > "$OUT/bench.log" 2>&1 || exit $?
tail -1 "$OUT/bench.log" | cut -c1-600
