#!/bin/bash
# Round-5 GPU session: the new GPU tests (+ an optional test list), a kernel trace of the graphed PPO
# collect (512-step horizon), then the configs[2] (65536 x 2048) and configs[4] (262144 x 1000) legs.
# Usage: tools/r05_session.sh TAG [pytest targets...]; every GPU step has its own time limit and the
# script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
TAG=${1:-r05}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
TESTS=${*:-tests/test_gpu_r05.py tests/test_gpu_r04.py}
timeout -k 10 500 python -u -m pytest $TESTS -x -v --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
[ -n "$SKIP_PROF" ] && exit 0
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ctrace" -- \
  python3 bench.py --rollout-steps 512 --sac-fill-steps 0 --no-cpu-baseline --no-open-loop --long-window 0 --no-fp64 \
  --no-replay --steps 20 --warmup 2 --prep 100 > "$OUT/collect512.log" 2>&1 || exit $?
find "$OUT/ctrace" -name "*kernel_stats.csv" -exec cp {} "$OUT/collect_kernel_stats.csv" \;
head -12 "$OUT/collect_kernel_stats.csv" | cut -c1-160
timeout -k 10 500 python3 bench.py --no-cpu-baseline --no-open-loop --long-window 0 --no-fp64 --no-replay \
  --steps 5 --warmup 2 --prep 100 > "$OUT/legs.log" 2>&1 || exit $?
tail -1 "$OUT/legs.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'rollout': d.get('rollout'), 'sac_fill': d.get('sac_fill')}))"
