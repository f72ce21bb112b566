#!/bin/bash
# Round-4 profiling session: (1) kernel trace of the graphed PPO collect (512-step horizon), (2) the
# configs[2] collect rate at its 2048 horizon, (3) the k_env_step HBM traffic split (no-reset vs steady).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-r04prof}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "$PROF_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $PROF_TESTS -x -q --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1
  rc=$?; tail -1 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ctrace" -- \
  python3 bench.py --rollout-steps 512 --no-cpu-baseline --no-open-loop --long-window 0 --no-fp64 --no-replay \
  --steps 20 --warmup 2 --prep 100 > "$OUT/collect512.log" 2>&1 || exit $?
find "$OUT/ctrace" -name "*kernel_stats.csv" -exec cp {} "$OUT/collect_kernel_stats.csv" \;
tail -1 "$OUT/collect512.log" | cut -c1-300
timeout -k 10 400 python3 bench.py --rollout-steps 2048 --no-cpu-baseline --no-open-loop --long-window 0 --no-fp64 \
  --no-replay --steps 5 --warmup 2 --prep 100 > "$OUT/collect2048.log" 2>&1 || exit $?
tail -1 "$OUT/collect2048.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('collect2048', d['rollout']['env_steps_per_s'], d['rollout']['collect_s'])"
[ -n "$SKIP_SPLIT" ] || bash tools/r04_traffic.sh "${1:-r04prof}_split"
