cd $GRAFT_REPO_ROOT
O=gpurun_out/r03h; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_r03.py -k teacher -v --timeout 300 --timeout-method thread -rf -s > $O/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "teacher-forced" $O/pytest.log | tail -3
