cd $GRAFT_REPO_ROOT
O=gpurun_out/r03k; mkdir -p $O
timeout -k 10 900 python -u tools/fp64_stuck.py 1300 20000 > $O/stuck.log 2>&1; rc=$?; echo stuck rc=$rc; grep device_nfev $O/stuck.log | head -6; tail -3 $O/stuck.log
