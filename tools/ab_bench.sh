#!/bin/bash
# A/B of library variants (tools/ab.py build NAME ...) on the bench line: closed-loop value and the
# open-loop rollout line per variant.  Usage: tools/ab_bench.sh NAME...   (GPU)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/ab
for v in "$@"; do
  FWSIM_LIB=tools/_build/variants/$v.so timeout -k 10 240 python bench.py --no-cpu-baseline --no-weak ${AB_ARGS} \
    > gpurun_out/ab/$v.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab/$v.log').read().strip().splitlines()[-1]); o=d.get('open_loop_rollout') or {}; print('$v', 'closed %.4g (%.4f ms)' % (d['value'], d['ms_per_step']), 'open %.4g (%.4f ms)' % (o.get('value', 0), o.get('ms_per_step', 0)), 'early %.4f ms' % d['early_regime']['kernel_ms'])"
done
