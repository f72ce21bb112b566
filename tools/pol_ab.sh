#!/bin/bash
# A/B of the policy-launch variant: its rollout tests, then the collect profile, both on FWSIM_LIB.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-polab}
mkdir -p "$OUT"
export FWSIM_LIB=$PWD/tools/_build/variants/rowpf.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_r02.py::test_graphed_collect_equals_eager -m gpu -x -q \
  --timeout 300 --timeout-method thread -rf > "$OUT/pytest.log" 2>&1 || { tail -5 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
bash tools/collect_prof.sh "${1:-polab}_prof"
