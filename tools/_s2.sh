cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03b
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/nfev_census.py 4000 gpurun_out/r03b/nfev_census.json > gpurun_out/r03b/census.log 2>&1; rc=$?; echo census rc=$rc; tail -3 gpurun_out/r03b/census.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_r03.py -x -v --timeout 300 --timeout-method thread -rf > gpurun_out/r03b/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -5 gpurun_out/r03b/pytest.log; [ $rc -le 1 ] || exit $rc
