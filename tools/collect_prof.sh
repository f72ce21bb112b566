#!/bin/bash
# Kernel-level breakdown of the graphed PPO collect (configs[2] shape, 65536 envs, 2048-step horizon: the bench leg).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-cprof}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -- \
  python3 bench.py --rollout-steps 2048 --sac-fill-steps 0 --no-cpu-baseline --no-open-loop --long-window 0 --no-fp64 --no-replay \
  --steps 20 --warmup 2 --prep 100 > "$OUT/bench.log" 2>&1 || exit $?
find "$OUT/trace" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
head -40 "$OUT/kernel_stats.csv" | cut -c1-220
tail -1 "$OUT/bench.log" | cut -c1-400
