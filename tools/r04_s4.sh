#!/bin/bash
# Driver-default bench on the current build, then the two-waves-per-SIMD A/B (tools/r04_waves.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-s4}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1 || exit $?
tail -1 "$OUT/bench.log" | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); w=d['window']['timed']
print('value', d['value'], 'ms', d['ms_per_step'], 'long', d['long_window']['kernel_ms'], 'fp64', d['fp64']['long_window']['kernel_ms'], 'collect', d['rollout']['env_steps_per_s'])
print('max_nfev', w['max_nfev'], w['slowest_launches'][:3])"
[ -n "$SKIP_WAVES" ] || bash tools/r04_waves.sh "${1:-s4}_waves"
