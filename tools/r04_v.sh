# round-4 call v: the driver's round-end checks on the final tree (GPU suite, smoke, default bench)
mkdir -p gpurun_out/v
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/v/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/v/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/v/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/v/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/v/bench.log | cut -c1-400; exit $rc
