#!/bin/bash
# Round-4 check after an RHS change: GPU suite, lone-wave tail fit, the driver-default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-s5}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
  || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 200 python3 tools/tail.py > "$OUT/tail.log" 2>&1 || exit $?
tail -2 "$OUT/tail.log" | head -1 | cut -c1-400
SKIP_WAVES=1 bash tools/r04_s4.sh "${1:-s5}"
