set -e
O=gpurun_out/ab3; mkdir -p $O
for v in cur np64; do
  FWSIM_LIB=tools/_build/variants/$v.so TAIL_PREC=float64 TAIL_N=8192 TAIL_STEPS=200 timeout -k 10 300 python -u tools/tail.py > $O/$v.log 2>&1
  grep "{" $O/$v.log | head -1
done
FWSIM_LIB=tools/_build/variants/cur.so ROLL_PREC=float64 timeout -k 10 300 python -u tools/rollout_probe.py >> $O/probe.log 2>&1
