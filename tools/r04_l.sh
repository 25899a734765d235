# round-4 call l: STRICT FFT / AUTO at default three-pass geometry (2^25..2^27)
mkdir -p gpurun_out/l && timeout -k 10 600 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_modwt_strict_gpu.py -k "default_geometry or auto_2_25" > gpurun_out/l/pytest_long.log 2>&1; rc=$?; tail -8 gpurun_out/l/pytest_long.log; exit $rc
