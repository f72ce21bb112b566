#!/bin/bash
# Round-6 session 8: the open loop with y / f back in LDS for k_env_rollout only (template YF = false) against the
# all-LDS variant (tools/_build/ab/noyf.so), alternated; then the whole GPU suite (rollout == K env steps bit for bit).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-r06s8}
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in 1 2; do
  ROLL_PREC=float32 ROLL_N=65536 ROLL_K=256 ROLL_LAUNCHES=16 ROLL_PREP=1000 ROLL_PREP_MODE=open \
    timeout -k 10 300 python tools/rollout_probe.py > "$OUT/tree_$r.log" 2>&1 || exit $?
  tail -1 "$OUT/tree_$r.log"
  FWSIM_LIB=tools/_build/ab/noyf.so ROLL_PREC=float32 ROLL_N=65536 ROLL_K=256 ROLL_LAUNCHES=16 ROLL_PREP=1000 \
    ROLL_PREP_MODE=open timeout -k 10 300 python tools/rollout_probe.py > "$OUT/noyf_$r.log" 2>&1 || exit $?
  tail -1 "$OUT/noyf_$r.log"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1 || exit $?
tail -1 "$OUT/bench.log" | cut -c1-200
