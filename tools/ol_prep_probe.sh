#!/bin/bash
# Open-loop rate vs how the population was prepared and how many launches are timed (fp32, 65536, K = 256).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-olp}
mkdir -p "$OUT"
for mode in open closed; do
  for L in 4 8 16; do
    ROLL_PREC=float32 ROLL_N=65536 ROLL_K=256 ROLL_LAUNCHES=$L ROLL_PREP=1000 ROLL_PREP_MODE=$mode \
      timeout -k 10 300 python tools/rollout_probe.py 2>/dev/null | grep '^{' >> "$OUT/prep.log" || exit $?
  done
done
cat "$OUT/prep.log"
