#!/bin/bash
# Is the steady window's extra HBM traffic per done aircraft?  FETCH/WRITE per k_env_step dispatch with the
# default episode length and with steps_max = 50 (every aircraft resets every 50 steps).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-split2}
mkdir -p "$OUT"
export TMPDIR=/tmp
for cfg in default:: sm50:50; do
  name=${cfg%%:*}; sm=${cfg#*:}; sm=${sm#:}
  for ctr in FETCH_SIZE WRITE_SIZE; do
    SPLIT_STEPS_MAX=$sm SPLIT_PREP=300 timeout -k 10 240 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/${name}_$ctr" -- \
      python3 tools/traffic_split.py > "$OUT/${name}_$ctr.log" 2>&1 || exit $?
    echo "$name $ctr ok"
  done
done
