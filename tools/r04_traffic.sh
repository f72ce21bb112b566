#!/bin/bash
# HBM traffic split of k_env_step (no-reset window vs steady window), FETCH_SIZE / WRITE_SIZE in separate
# rocprofv3 passes (MI355X guide recipe), calibrated on tools/fetch_calib.hip.  -> profiles/r04_traffic_split.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-split}
mkdir -p "$OUT" tools/_build
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 "$OUT/$name.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
[ -x tools/_build/fetch_calib ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o tools/_build/fetch_calib tools/fetch_calib.hip || exit 3
step calib_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/calib_fetch" -- tools/_build/fetch_calib
step calib_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/calib_write" -- tools/_build/fetch_calib
step split_fetch 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/split_fetch" -- python3 tools/traffic_split.py
step split_write 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/split_write" -- python3 tools/traffic_split.py
python3 tools/traffic_split_report.py "$OUT"
