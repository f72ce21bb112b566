#!/bin/bash
# configs[2] collect (65536 x 2048) with 16 / 32 / 64 collect steps per graph replay (RolloutCollector.steps_per_graph).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/spg
for K in 16 32 64; do
  timeout -k 10 300 python3 -c "
import sys, runpy
sys.argv = ['bench.py', '--rollout-steps', '2048', '--no-cpu-baseline', '--no-open-loop', '--long-window', '0', '--no-fp64', '--no-replay', '--steps', '5', '--warmup', '2', '--prep', '100']
from tum_adlr_deep_reinforcement_learning_amd.rollout import RolloutCollector
RolloutCollector.steps_per_graph = $K
runpy.run_path('bench.py', run_name='__main__')
" > gpurun_out/spg/k$K.log 2>&1 || exit $?
  tail -1 gpurun_out/spg/k$K.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('K=$K', d['rollout']['env_steps_per_s'], d['rollout']['host_launches_per_step'])"
done
