#!/bin/bash
# The driver's bench command profiled: a kernel trace (per-launch durations of the 20 timed launches) and
# the PMC passes (HBM bytes, VALU instructions) over the same 20 launches.  GPU; outputs under
# gpurun_out/$TAG/.  Usage: TAG=r03i bash tools/r03_profile.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/${TAG:-r03i}; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 "$O/$name.log"; [ $rc -eq 0 ] || exit $rc; }
step trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
python3 tools/driver_window.py $O/trace 20 5 1000 $O/driver_window.json
cp $(find $O/trace -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv 2>/dev/null
# PMC over the same 20 launches: nothing after the timed window (no long window / replay / legs)
export BENCH_ARGS="--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --long-window 0 --no-open-loop --no-fp64 --no-replay"
export PMC_LAST=20 PMC_WINDOW="the 20 timed dispatches of the driver's command (bench.py --steps 20 --warmup 5)"
bash tools/traffic.sh > $O/traffic.log 2>&1; rc=$?; echo traffic rc=$rc; tail -2 $O/traffic.log; [ $rc -eq 0 ] || exit $rc
cp gpurun_out/traffic/pmc_env_step.json $O/
step bench 400 python3 bench.py --gpus 1 --steps 20 --warmup 5
