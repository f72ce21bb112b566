#!/bin/bash
# HBM traffic of k_env_step from PMC counters, per the MI355X guide's recipe:
# FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes (they do not fit one
# pass), --pmc never combined with sys/runtime traces, and the unit/width
# correction calibrated on tools/fetch_calib.hip (same 4-B/lane SoA pattern).
# Output: gpurun_out/traffic/*.csv and profiles/pmc_env_step.json (via traffic_report.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/traffic tools/_build
export TMPDIR=/tmp
BENCH_ARGS=${BENCH_ARGS:-"--steps 200 --warmup 16 --no-cpu-baseline --long-window 0 --no-open-loop"}
step() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > "gpurun_out/traffic/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 "gpurun_out/traffic/$name.log"; [ $rc -eq 0 ] || exit $rc; }
[ -x tools/_build/fetch_calib ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o tools/_build/fetch_calib tools/fetch_calib.hip || exit 3
step calib_fetch 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/traffic/calib_fetch -- tools/_build/fetch_calib
step calib_write 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/traffic/calib_write -- tools/_build/fetch_calib
step env_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/traffic/env_fetch -- python bench.py $BENCH_ARGS
step env_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/traffic/env_write -- python bench.py $BENCH_ARGS
step env_valu 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/traffic/env_valu -- python bench.py $BENCH_ARGS
python tools/traffic_report.py gpurun_out/traffic
