#!/bin/bash
# fp64 closed loop at 65536 aircraft: one lane + tail handoff (automatic) vs lane quads for every aircraft.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-fp64lanes}
mkdir -p "$OUT"
for L in 0 4; do
  timeout -k 10 300 python3 bench.py --precision float64 --lanes $L --steps 20 --warmup 5 --no-cpu-baseline \
    --no-open-loop --rollout-steps 0 --no-replay --no-fp64 > "$OUT/lanes$L.log" 2>&1 || exit $?
  tail -1 "$OUT/lanes$L.log" | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('lanes $L', 'window', d['ms_per_step'], 'early', d['early_regime']['kernel_ms'], 'long', d['long_window']['kernel_ms'])"
done
