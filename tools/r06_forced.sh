#!/bin/bash
# Round-6: the whole GPU suite with each integrator forced (FWSIM_LANES=1 / 2 / 4) on the final build; the tests of
# the automatic lanes choice skip themselves under the override.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-r06forced}
mkdir -p "$OUT"
export TMPDIR=/tmp
for L in 1 4 2; do
  FWSIM_LANES=$L timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf \
    > "$OUT/lanes$L.log" 2>&1
  rc=$?; echo "lanes $L: $(tail -1 "$OUT/lanes$L.log")"; [ $rc -le 1 ] || exit $rc
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > "$OUT/auto.log" 2>&1
rc=$?; echo "auto: $(tail -1 "$OUT/auto.log")"; exit $rc
