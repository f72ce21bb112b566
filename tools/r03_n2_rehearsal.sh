#!/bin/bash
# Rehearsal of bench.py's N > 1 path on a one-GPU box: two ranks, both on cuda:0, gloo backend
# (RCCL refuses two ranks on one device).  Checks that every leg of the N > 1 line runs and prints;
# the numbers are not a scaling measurement (the two ranks share one GPU).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-r03n2}
mkdir -p "$OUT"
FW_BENCH_ONE_DEVICE=1 FW_BENCH_BACKEND=gloo timeout -k 10 700 python bench.py --gpus 2 --steps 20 --warmup 5 \
  > "$OUT/bench_n2.log" 2>&1
rc=$?
echo "bench_n2 rc=$rc"; tail -2 "$OUT/bench_n2.log" | cut -c1-600
exit $rc
