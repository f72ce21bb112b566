(for i in $(seq 1 40); do date +%s.%N; rocm-smi --showclocks --showpower 2>/dev/null | grep -E "sclk|Power|fclk" ; sleep 0.5; done) > gpurun_out/smi.log 2>&1 &
SMI=$!
timeout -k 10 120 python tools/drift_probe.py 65536 1500 > gpurun_out/drift_a.log 2>&1
timeout -k 10 120 python tools/drift_probe.py 65536 1000 0.3 > gpurun_out/drift_b.log 2>&1
kill $SMI
