#!/bin/bash
# Counter A/B, one-lane (+ tail handoff) vs pair, k_env_step at 65536 and 32768 aircraft (identical states).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-r06pairpmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
K=40
for N in 65536 32768; do
  for L in 1 2; do
    i=0
    for set in "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_LDS" \
               "SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SMEM SQ_INSTS_SALU SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM"; do
      i=$((i+1))
      d="$OUT/n${N}_l${L}_p$i"
      timeout -k 10 -s KILL 240 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$d" -- python tools/pair_pmc.py $N $L $K 300 > "$d.log" 2>&1
      rc=$?; [ $rc -le 1 ] || { echo "pass rc=$rc"; tail -5 "$d.log"; exit $rc; }
    done
    python tools/pair_pmc_report.py "$OUT" $L $K > /dev/null  # (sanity)
    python - "$OUT" $N $L $K <<'PY'
import collections, csv, glob, json, os, sys
root, N, L, K = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
tag = "Li%dE" % L
cnt = collections.defaultdict(dict)
dur = []
for f in sorted(glob.glob(os.path.join(root, "n%d_l%d_p*" % (N, L), "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        if "k_env_step" in r["Kernel_Name"] and tag in r["Kernel_Name"]:
            d = (f, int(r["Dispatch_Id"]))
            cnt[r["Counter_Name"]][d] = cnt[r["Counter_Name"]].get(d, 0.0) + float(r["Counter_Value"])
for f in sorted(glob.glob(os.path.join(root, "n%d_l%d_p1" % (N, L), "**", "*kernel_trace.csv"), recursive=True)):
    rows = [r for r in csv.DictReader(open(f)) if "k_env_step" in r["Kernel_Name"] and tag in r["Kernel_Name"]]
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows][-K:]
res = {}
for c, dv in cnt.items():
    ks = sorted(dv)[-K:]
    res[c] = sum(dv[k] for k in ks) / len(ks)
print(json.dumps({"envs": N, "lanes": L, "launch_us_mean_profiled": sum(dur) / max(len(dur), 1), "counters": res}))
PY
  done
done
