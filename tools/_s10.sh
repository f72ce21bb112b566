set -e
O=gpurun_out/ol; mkdir -p $O
ROLL_PREC=float32 ROLL_K=256 ROLL_LAUNCHES=4 ROLL_PREP=1000 timeout -k 10 300 python -u tools/rollout_probe.py >> $O/probe.log 2>&1
ROLL_PREC=float32 ROLL_K=1024 ROLL_LAUNCHES=1 ROLL_PREP=1000 timeout -k 10 300 python -u tools/rollout_probe.py >> $O/probe.log 2>&1
ROLL_PREC=float32 ROLL_K=64 ROLL_LAUNCHES=16 ROLL_PREP=1000 timeout -k 10 300 python -u tools/rollout_probe.py >> $O/probe.log 2>&1
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-fp64 > $O/bench.json 2> $O/bench.err
