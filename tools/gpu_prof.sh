#!/bin/bash
# profiling session: sweep + rocprofv3 kernel trace + one PMC pass
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -12 "gpurun_out/$name.log"; [ $rc -le 1 ] || exit $rc; }
step sweep 300 python tools/sweep.py
step sweep64 300 python tools/sweep.py --precision float64 --sizes 4096,65536 --steps 5
step rocprof_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_trace -- python bench.py --steps 100 --warmup 10 --no-cpu-baseline
step rocprof_pmc 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/prof_pmc -- python tools/sweep.py --sizes 65536 --steps 3
