# round-4 call u: sym8 forward at five waves per SIMD (variant fwd5): parity and A/B
mkdir -p gpurun_out/u
JWAVE_HIP_LIB=$PWD/jwave-pro_amd/ab/libjwave_hip_fwd5.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_modwt_gpu.py > gpurun_out/u/pytest_fwd5.log 2>&1; rc=$?; tail -1 gpurun_out/u/pytest_fwd5.log; [ $rc -eq 0 ] || exit $rc
REPS="1 2 3" STEPS=10 bash tools/ab_modwt_libs.sh u fwd5
