cd $GRAFT_REPO_ROOT
O=gpurun_out/r03e; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/_diag_quad.py > $O/diag.log 2>&1; rc=$?; echo diag rc=$rc; cat $O/diag.log | tail -14; [ $rc -le 1 ] || exit $rc
timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rf --deselect "tests/test_gpu_quad.py::test_quad_stragglers[float64]" > $O/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -8 $O/pytest.log; [ $rc -le 1 ] || exit $rc
