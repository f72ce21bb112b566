#!/bin/bash
# Open-loop rollout steps-per-launch sweep (fp32, 65536 aircraft, 2048 timed steps per K).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-olk}
mkdir -p "$OUT"
for K in 128 256 512 1024; do
  ROLL_PREC=float32 ROLL_N=65536 ROLL_K=$K ROLL_LAUNCHES=$((2048 / K)) ROLL_PREP=1000 \
    timeout -k 10 300 python tools/rollout_probe.py >> "$OUT/ksweep.log" 2>&1 || exit $?
done
cat "$OUT/ksweep.log"
