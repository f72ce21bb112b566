#!/bin/bash
# Profiles behind bench.py's line: PMC traffic + VALU passes (tools/traffic.sh), the rocprofv3 kernel
# trace of the default bench with its timed-window summary, then the bench itself with the CPU baseline.
# Usage: tools/prof_session.sh TAG     (outputs under gpurun_out/TAG/)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
TAG=${1:-prof}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/traffic.sh > "$OUT/traffic.log" 2>&1; rc=$?; echo "traffic rc=$rc"; tail -3 "$OUT/traffic.log"; [ $rc -eq 0 ] || exit $rc
cp gpurun_out/traffic/pmc_env_step.json "$OUT/"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -- python bench.py --no-cpu-baseline --long-window 0 --no-open-loop \
  > "$OUT/trace.log" 2>&1; rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
python tools/trace_window.py "$OUT/trace" 200 k_env_step "$OUT/trace_window.json"
timeout -k 10 300 python bench.py > "$OUT/bench.log" 2>&1; rc=$?; echo "bench rc=$rc"; tail -c 3000 "$OUT/bench.log"; exit $rc
