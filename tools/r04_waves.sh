#!/bin/bash
# Second resident wave per SIMD at 65536 aircraft: the one-lane k_env_step instances at __launch_bounds__(64, 2)
# (tools/ab.py build mw2 -DFW_MIN_WAVES=2) against the shipped one-wave build -- bench A/B (two repetitions)
# and SQ counters over the driver's 20 timed dispatches of each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
TAG=${1:-waves}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
AB_SIZES=65536 bash tools/ab_lanes.sh "$TAG" default tools/_build/variants/mw2.so || exit $?
BENCH_ARGS="--steps 20 --warmup 5 --no-cpu-baseline --long-window 0 --no-open-loop --no-fp64 --no-replay --rollout-steps 0 --no-weak"
for v in default mw2; do
  L=; [ "$v" = mw2 ] && L=tools/_build/variants/mw2.so
  i=0
  for set in "SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_SALU" \
             "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM"; do
    i=$((i+1))
    FWSIM_LIB=$L timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d "$OUT/pmc_${v}_$i" -- \
      python3 bench.py $BENCH_ARGS > "$OUT/pmc_${v}_$i.log" 2>&1
    rc=$?; echo "pmc $v $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
python3 - "$OUT" <<'PY'
import csv, glob, json, os, sys
base = sys.argv[1]
res = {}
for v in ("default", "mw2"):
    per = {}
    for f in glob.glob(os.path.join(base, "pmc_%s_*" % v, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_env_step<float" in r["Kernel_Name"]:
                per.setdefault(r["Counter_Name"], {}).setdefault(int(r["Dispatch_Id"]), 0.0)
                per[r["Counter_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    res[v] = {k: sum(sorted(d.items())[-20:][i][1] for i in range(min(20, len(d)))) / min(20, len(d)) for k, d in per.items()}
print(json.dumps(res))
open(os.path.join(base, "waves_pmc.json"), "w").write(json.dumps(res, indent=1))
PY
