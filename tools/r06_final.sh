#!/bin/bash
# Round-6 evidence session on the committed tree: N = 2 rehearsal (gloo, one device), smoke, the GPU suite, the
# driver's bench command (plain, then under a kernel trace for the driver window), the PMC passes of the driver
# window (refreshes profiles/pmc_env_step.json for the bench line's roofline.traffic) and the kernel breakdown of
# the fused PPO collect (configs[2] shape).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-r06final}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -z "$SKIP_N2" ]; then bash tools/r03_n2_rehearsal.sh "$(basename $OUT)_n2" || exit $?; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
tail -1 "$OUT/smoke.log"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > "$OUT/pytest.log" 2>&1
  rc=$?; tail -1 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1 || exit $?
tail -1 "$OUT/bench.log" | cut -c1-300
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_traced.log" 2>&1 || exit $?
find "$OUT/trace" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
python3 tools/driver_window.py "$OUT/trace" 20 5 1000 "$OUT/driver_window.json" | cut -c1-300
BENCH_ARGS="--steps 20 --warmup 5 --no-cpu-baseline --long-window 0 --no-open-loop --no-fp64 --no-replay --rollout-steps 0 --sac-fill-steps 0" PMC_LAST=20 \
  PMC_WINDOW="the driver's window: bench.py --steps 20 --warmup 5 (the last 20 k_env_step dispatches of the timed engine)" \
  bash tools/traffic.sh || exit $?
cp profiles/pmc_env_step.json "$OUT/pmc_env_step.json"
bash tools/collect_prof.sh "$(basename $OUT)_collect" || exit $?
# fp64 vs fp32 one-lane env step counters over the same tail protocol (40 launches)
for prec in float32 float64; do
  TAIL_PREC=$prec TAIL_STEPS=40 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d "$OUT/pmc_$prec" -- python3 tools/tail.py > "$OUT/pmc_$prec.log" 2>&1 || exit $?
done
