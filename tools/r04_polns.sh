#!/bin/bash
# (The net-split kernel was not adopted and is no longer in fw_rollout.hip; profiles/r04_ab_collect.log has the result.)
# Net-split policy kernel (k_policy_mfma_ns) vs the two-net kernel (FW_POL_NS=0): standalone launch time,
# the policy / collect GPU tests, and the collect legs (64-step bench leg and configs[2] 2048).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-polns}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/pol_bench.py > "$OUT/pol_ns.log" 2>&1 || exit $?
FW_POL_NS=0 timeout -k 10 120 python3 tools/pol_bench.py > "$OUT/pol_2net.log" 2>&1 || exit $?
echo "ns $(grep kernel "$OUT/pol_ns.log")"; echo "2net $(grep kernel "$OUT/pol_2net.log")"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "policy or collect or rollout or vecnorm or merge" --timeout 200 \
  --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for v in 1 0; do
  FW_POL_NS=$v timeout -k 10 400 python3 bench.py --rollout-steps 2048 --no-cpu-baseline --no-open-loop --long-window 0 \
    --no-fp64 --no-replay --steps 5 --warmup 2 --prep 100 > "$OUT/collect2048_$v.log" 2>&1 || exit $?
  tail -1 "$OUT/collect2048_$v.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ns=$v collect2048', d['rollout']['env_steps_per_s'])"
done
