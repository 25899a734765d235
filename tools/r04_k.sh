# round-4 call k: wave2 inverse loads with uniform (SGPR) row offsets: MODWT parity, then A/B
mkdir -p gpurun_out/k && timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_modwt_gpu.py tests/test_modwt_strict_gpu.py > gpurun_out/k/pytest_modwt.log 2>&1 && tail -2 gpurun_out/k/pytest_modwt.log && bash tools/ab_modwt_libs.sh k soff0
