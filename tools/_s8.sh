cd $GRAFT_REPO_ROOT
O=gpurun_out/r03j; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_r02.py -k "rollout or offpolicy or c5" -v --timeout 300 --timeout-method thread -rf > $O/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -3 $O/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-fp64 --no-replay > $O/bench.json 2> $O/bench.err; rc=$?; echo bench rc=$rc; [ $rc -eq 0 ] || exit $rc
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['long_window'],d['open_loop_rollout'])"
timeout -k 10 500 python -u tools/fp64_stuck.py 480 20000 > $O/stuck.log 2>&1; rc=$?; echo stuck rc=$rc; grep device_nfev $O/stuck.log | head -6; tail -2 $O/stuck.log
