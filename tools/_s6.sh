cd $GRAFT_REPO_ROOT
O=gpurun_out/r03g; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rf -s > $O/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "teacher-forced|passed|failed" $O/pytest.log | tail -6; [ $rc -le 1 ] || exit $rc
TAIL_STEPS=400 timeout -k 10 200 python -u tools/tail.py > $O/tail.log 2>&1; rc=$?; echo tail rc=$rc; head -1 $O/tail.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-fp64 > $O/bench.json 2> $O/bench.err; rc=$?; echo bench rc=$rc; [ $rc -eq 0 ] || exit $rc
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['long_window'],d['open_loop_rollout']['value'],d['window']['timed']['launch_ms'])"
timeout -k 10 200 python -u tools/fp64_probe.py 200 240 > $O/fp64.log 2>&1; rc=$?; echo fp64 rc=$rc; tail -1 $O/fp64.log; [ $rc -eq 0 ] || exit $rc
FWSIM_TAIL_QUAD=0 timeout -k 10 200 python -u tools/fp64_probe.py 200 240 > $O/fp64_noho.log 2>&1; rc=$?; echo fp64 noho rc=$rc; tail -1 $O/fp64_noho.log
