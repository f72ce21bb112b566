#!/bin/bash
# Round-6 session 7: the open-loop leg (fw_env_rollout, 65536 x 256-step launches) with the accepted y / f in
# registers (in-tree, FW_YF_REGS=1) vs in LDS (tools/_build/ab/noyf.so), alternated, identical states.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-r06s7}
mkdir -p "$OUT"
for r in 1 2; do
  ROLL_PREC=float32 ROLL_N=65536 ROLL_K=256 ROLL_LAUNCHES=16 ROLL_PREP=1000 ROLL_PREP_MODE=open \
    timeout -k 10 300 python tools/rollout_probe.py > "$OUT/yf_$r.log" 2>&1 || exit $?
  tail -1 "$OUT/yf_$r.log"
  FWSIM_LIB=tools/_build/ab/noyf.so ROLL_PREC=float32 ROLL_N=65536 ROLL_K=256 ROLL_LAUNCHES=16 ROLL_PREP=1000 \
    ROLL_PREP_MODE=open timeout -k 10 300 python tools/rollout_probe.py > "$OUT/noyf_$r.log" 2>&1 || exit $?
  tail -1 "$OUT/noyf_$r.log"
done
