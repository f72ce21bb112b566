cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03c
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03c/bench_driver.json 2> gpurun_out/r03c/bench_driver.err; rc=$?; echo bench rc=$rc; tail -5 gpurun_out/r03c/bench_driver.err; [ $rc -eq 0 ] || exit $rc
