#!/bin/bash
# Round 6: the deferred final merge (fw_collect_epilogue.defer) -- its GPU tests, then the configs[2] collect leg
# (65536 envs x 2048 steps, bench.py's rollout leg) with the deferral on / off, alternated, and a kernel trace of
# each (k_env_step / k_policy_mfma averages inside the collect).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-r06collect}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -rf \
  tests/test_gpu_r06.py tests/test_gpu_r05.py tests/test_gpu_r04.py tests/test_gpu_rollout.py \
  > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
LEG="--rollout-steps 2048 --sac-fill-steps 0 --no-cpu-baseline --no-open-loop --long-window 0 --no-fp64 --no-replay --steps 20 --warmup 2 --prep 100"
for r in 1 2; do
  for d in 1 0; do
    FW_DEFER_FINAL_MERGE=$d timeout -k 10 300 python bench.py $LEG > "$OUT/leg_d${d}_$r.log" 2>&1 || exit $?
    python - "$OUT/leg_d${d}_$r.log" "$d" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["rollout"]
print(json.dumps({"defer": int(sys.argv[2]), "collect_env_steps_per_s": round(r["env_steps_per_s"]), "collect_s": round(r["collect_s"], 4),
                  "graph_kernel_nodes": r["graph_kernel_nodes"]}), flush=True)
PY
  done
done
for d in 1 0; do
  FW_DEFER_FINAL_MERGE=$d timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_d$d" -- \
    python3 bench.py $LEG > "$OUT/traced_d$d.log" 2>&1 || exit $?
  find "$OUT/trace_d$d" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats_d$d.csv" \;
  python3 - "$OUT/kernel_stats_d$d.csv" "$d" <<'PY'
import csv, json, sys
rows = list(csv.DictReader(open(sys.argv[1])))
out = {"defer": int(sys.argv[2])}
for r in rows:
    for k in ("k_env_step", "k_policy_mfma", "k_pending_update", "k_gae"):
        if k in r["Name"]:
            out[k] = {"calls": int(r["Calls"]), "avg_us": round(float(r["AverageNs"]) / 1e3, 2)}
print(json.dumps(out), flush=True)
PY
done
