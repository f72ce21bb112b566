#!/bin/bash
# (The 1024-thread merge was not adopted and is no longer in fw_rollout.hip; profiles/r04_ab_collect.log has the result.)
# 1024-thread merge (k_merge_update1k, default) vs the 256-thread merge (FW_MERGE1K=0): standalone launch times,
# the VecNormalize / collect GPU tests, and the configs[2] collect at 2048 with each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-merge1k}
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in 1 0; do
  FW_MERGE1K=$v timeout -k 10 120 python3 tools/merge_bench.py > "$OUT/mb_$v.log" 2>&1 || exit $?
  echo "merge1k=$v $(grep '{' "$OUT/mb_$v.log" | tail -3 | tr '\n' ' ')"
done
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "policy or collect or rollout or vecnorm or merge or moments or shard" \
  --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for v in 1 0; do
  FW_MERGE1K=$v timeout -k 10 400 python3 bench.py --rollout-steps 2048 --no-cpu-baseline --no-open-loop --long-window 0 \
    --no-fp64 --no-replay --steps 5 --warmup 2 --prep 100 > "$OUT/collect2048_$v.log" 2>&1 || exit $?
  tail -1 "$OUT/collect2048_$v.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('merge1k=$v collect2048', d['rollout']['env_steps_per_s'])"
done
